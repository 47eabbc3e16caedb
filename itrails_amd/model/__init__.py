"""Model build of the iTRAILS HMM on the GPU."""
from .trans_emiss import trans_emiss_calc  # noqa: F401
