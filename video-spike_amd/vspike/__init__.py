"""vspike — MI355X-native (gfx950) video->spike training hot path of PPWangyc/video-spike.

Drop-in surface (src/utils/utils.py:28-34 of the reference): `NAME2MODEL[config.model.model_class]`
builds the plugin from `config.model`; `forward(inputs) -> log-rates (B, 100, N)`.  All compute
runs in libvspike.so (hand-written HIP, include/vspike.h) — there is no CPU fallback.
"""
from .config import DictConfig, config_from_kwargs, load_run_config, update_config
from .linear import Linear
from .loss import MSEMeanLoss, PoissonNLLMeanLoss, make_criterion, mse_mean, poisson_nll_mean
from .optim import FusedAdamW
from .r3d import R3D
from .vit import VideoMAE

NAME2MODEL = {
    "Linear": Linear,
    "VideoMAE": VideoMAE,
    # BASELINE C4's CNN encoder (no reference counterpart: SURVEY.md section 0), same plugin surface
    "R3D": R3D,
}

__all__ = ["NAME2MODEL", "Linear", "VideoMAE", "R3D", "FusedAdamW", "poisson_nll_mean", "PoissonNLLMeanLoss",
           "mse_mean", "MSEMeanLoss", "make_criterion",
           "DictConfig", "update_config", "config_from_kwargs", "load_run_config"]
