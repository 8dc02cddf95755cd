"""MI355X-native NeRF ray-march hot path (gfx950 HIP kernels behind a C ABI).

  ops       tensor-level wrappers of the C ABI (encoders + step kernels)
  fused     FusedRenderer: NeRFRenderer.run as five fused kernel launches
  dist      ray sharding over ranks + RCCL all-gather of output tiles
"""
from ._lib import EXPORTED, LIB_PATH, SamnerfUnavailable, lib  # noqa: F401
