"""In-sample optimisers whose likelihood evaluations run batched on the device
(SURVEY.md §8f ranks 2-3): the reference's optimiser control flow, with every
likelihood the optimiser needs for one step gathered into one device launch.

* garch.GarchOptimizer          garch/opti.py (Newton-Raphson + BIC order search)
* msm.Optimizer                 markov_switching_multifractal/opti.py (basin hopping, b sweep)
* copula_fit.Optimizer          copulas/student/opti.py (IFM, device t.ppf)
* copula_fit.GaussianCopulaOptimizer, PlackettCopulaOptimizer
"""
