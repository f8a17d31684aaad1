"""Import shim: ``from correlation_package.modules.correlation import Correlation`` (model.py:8
of the reference) resolves to the gfx950 implementation when pwc-net_pytorch_amd/ is on
sys.path ahead of the reference tree."""
