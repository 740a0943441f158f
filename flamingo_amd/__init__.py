"""flamingo_amd -- MI355X-native engine for Flamingo's per-round mask-and-aggregate path.

The package holds what the path needs and nothing else:
  csrc/      gfx950 HIP kernels + host runtime + C ABI (include/flamingo_hip.h)
  lib/       the built libflamingo_hip.so (in-tree, never a JIT cache)
  engine     ctypes handle on the library (host and device-resident calls)
  params     the reference's protocol constants and host-side graph logic
  distributed  the multi-GPU round (client-sharded rows, RCCL reduce-scatter)
  abides/    the ABIDES Kernel/Agent/Message surface and the Flamingo agents
"""
from .engine import DeviceGroup, MaskEngine, PinnedArena  # noqa: F401

__all__ = ["DeviceGroup", "MaskEngine", "PinnedArena"]
