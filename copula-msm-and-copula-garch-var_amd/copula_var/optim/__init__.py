"""In-sample optimisers whose likelihood evaluations run batched on the device
(SURVEY.md §8f rank 2): the reference's optimiser control flow, with every
likelihood the optimiser needs for one step gathered into one device launch."""
