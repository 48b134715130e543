"""sbce — MI355X-native EM semi-blind channel estimation for MIMO-RIS links.

Drop-in for the EM estimator path of
jrnerupudinho/Semi-Blind-Channel-Estimation-for-MIMO-RIS-communication-system-Using-EM-Algo:
the reference's ``em(...)`` operator ("Proposed method/Proposed_method_NMSEvsTp.py":50-83)
runs as hand-written HIP kernels for gfx950 behind the C-ABI of include/sbce.h.
"""
from . import _lib, qam, signal_model, layout, distributed  # noqa: F401
from . import sweeps  # noqa: F401
from ._lib import SbceUnavailable, SbceError  # noqa: F401
from .em import (  # noqa: F401
    em, em_ml, em_llf, em_ml_llf, em_ml_ser, em_pm, em_pm_soft, em_zf, em_mmse, em_superimposed,
    em_zero_init, em_batch, ser_batch, estep_batch,
    mstep_batch, nmse_batch, EMEngine, EM_Gaussian_proposed, gauss_expand_batch,
    gaussian_regressors, reduce_gaussian_channel,
)

__all__ = ["em", "em_ml", "em_llf", "em_ml_llf", "em_ml_ser", "em_pm", "em_pm_soft", "em_zf",
           "em_mmse", "em_superimposed", "ser_batch", "EM_Gaussian_proposed", "gauss_expand_batch",
           "em_zero_init", "em_batch",
           "SbceUnavailable", "SbceError", "qam", "signal_model"]
