"""acinoset_amd — MI355X-native (gfx950) core for AcinoSet's SBA / FTE hot path.

Drop-in Python entry points with the reference's signatures live in
`acinoset_amd.lib` (mirrors src/lib: sba, calib, misc, utils, metric, app) and
`acinoset_amd.core` (mirrors src/core: sba, fte, tri). All numeric work on the hot path
runs in hand-written HIP kernels behind the C ABI of include/acinoset_hip.h
(libacinoset_hip.so, loaded by `acinoset_amd._native`); there is no CPU fallback.
"""
__version__ = '0.1.0'
