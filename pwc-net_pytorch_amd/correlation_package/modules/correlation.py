"""correlation_package/modules/correlation.py drop-in (reference lines 6-27)."""
from pwcnet_amd.layers import Correlation

__all__ = ["Correlation"]
