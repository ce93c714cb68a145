"""(copula x model) factory -- utils/factory.py:10-31 of the reference, including
Q17: ('mean_reverting', 'gaussian') maps to the Plackett adapter (factory.py:22-23)."""
from .model_estimation.copula.gaussian_estimation import GaussianCopulaVaR
from .model_estimation.copula.plackett_estimation import PlackettCopulaVaR
from .model_estimation.copula.student_estimation import StudentCopulaVaR
from .model_estimation.model.garch_estimation import GarchEstimation
from .model_estimation.model.mean_reverting_estimation import MeanRevertingEstimation
from .model_estimation.model.msm_estimation import MSMEstimation

_TABLE = {
    ("msm", "student"): (StudentCopulaVaR, MSMEstimation),
    ("garch", "student"): (StudentCopulaVaR, GarchEstimation),
    ("mean_reverting", "student"): (StudentCopulaVaR, MeanRevertingEstimation),
    ("msm", "gaussian"): (GaussianCopulaVaR, MSMEstimation),
    ("garch", "gaussian"): (GaussianCopulaVaR, GarchEstimation),
    ("mean_reverting", "gaussian"): (PlackettCopulaVaR, MeanRevertingEstimation),     # Q17
    ("msm", "plackett"): (PlackettCopulaVaR, MSMEstimation),
    ("garch", "plackett"): (PlackettCopulaVaR, GarchEstimation),
    ("mean_reverting", "plackett"): (PlackettCopulaVaR, MeanRevertingEstimation),
}


class ValueAtRiskCalculationFactory:
    @staticmethod
    def create_var_calculator(copula_type, estimation_type):
        try:
            adapter, model = _TABLE[(estimation_type, copula_type)]
        except KeyError:
            raise ValueError("Unsupported estimation type.") from None
        return adapter(model())
