"""pwcnet_amd — MI355X (gfx950) hot path of PWC-Net: correlation, cost volume, flow warp.

Drop-in surface (reference daigo0927/PWC-Net_pytorch):
  Correlation, CorrelationFunction   <- correlation_package (modules/functions correlation.py)
  WarpingLayer, CostVolumeLayer       <- modules.py:25-74
  get_grid                            <- utils.py:3-8
The kernels live in libpwc_hotpath.so (C ABI: include/pwc_hotpath.h); there is no CPU path.
"""
from .layers import Correlation, CostVolumeLayer, WarpingLayer, get_grid
from .ops import CorrelationFunction, CostVolumeFunction, WarpFunction

__all__ = ["Correlation", "CorrelationFunction", "CostVolumeLayer", "CostVolumeFunction",
           "WarpingLayer", "WarpFunction", "get_grid"]
