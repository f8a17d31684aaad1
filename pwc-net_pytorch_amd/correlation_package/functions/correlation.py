"""correlation_package/functions/correlation.py drop-in (reference lines 7-56)."""
from pwcnet_amd.ops import CorrelationFunction

__all__ = ["CorrelationFunction"]
