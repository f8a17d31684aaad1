"""pwcnet_amd — MI355X (gfx950) hot path of PWC-Net: correlation, cost volume, flow warp.

Drop-in surface (reference daigo0927/PWC-Net_pytorch):
  Correlation, CorrelationFunction   <- correlation_package (modules/functions correlation.py)
  WarpingLayer, CostVolumeLayer       <- modules.py:25-74
  WarpCorrelation, WarpCorrelationFunction <- model.py:80-83 (warp then correlation, fused)
  UpsampleWarp, UpsampleWarpFunction  <- model.py:78 + :80 (flow upsample x2 then warp, fused)
  CorrelationCat, CorrelationCatFunction <- model.py:83-91 (corr [+ leaky_relu_] into the cat)
  get_grid                            <- utils.py:3-8
  flow_io.load_flow/save_flow/vis_flow <- flow_utils.py (.flo I/O + colour coding, numpy)
The kernels live in libpwc_hotpath.so (C ABI: include/pwc_hotpath.h); there is no CPU path.
"""
from .layers import (Correlation, CorrelationCat, CostVolumeLayer, UpsampleWarp,
                     WarpCorrelation, WarpingLayer, get_grid)
from .ops import (CorrelationCatFunction, CorrelationFunction, CostVolumeFunction,
                  UpsampleWarpFunction,
                  WarpCorrelationFunction, WarpFunction)

__all__ = ["Correlation", "CorrelationFunction", "CostVolumeLayer", "CostVolumeFunction",
           "WarpCorrelation", "WarpCorrelationFunction", "WarpingLayer", "WarpFunction",
           "UpsampleWarp", "UpsampleWarpFunction", "CorrelationCat", "CorrelationCatFunction",
           "get_grid"]
