from .base import BaseFlow  # noqa: F401
from .dynamics import LFIntegrator  # noqa: F401
from .loss import Alchemical_NLL  # noqa: F401
