"""mafrixraytracing_amd — MI355X-native path-tracing hot path for NAIVEddd/MafrixRaytracing.

Product layout:
  include/mafrix_rt.h          the C ABI (drop-in boundary for the F# Scene/Render API)
  csrc/                        HIP kernels for gfx950 + host scene/BVH preparation + the ABI
  libmafrix_rt.so              built by __graft_entry__.build() / `make -C csrc`
  abi.py                       ctypes mirror of the header (stands in for the F# P/Invoke layer)
  native.py                    Scene / NativePixelIntegrator / Film over the ABI
  scene_io.py                  Scene XML v0.1 + OBJ/MTL loading with the reference's semantics
  distributed.py               one-process-per-GPU sample partitioning + RCCL reduce
"""
from .abi import SceneArrays, load_library  # noqa: F401
from .scene_io import InitSceneState, MaterialManager, load_scene_file  # noqa: F401

__all__ = ["SceneArrays", "load_library", "InitSceneState", "MaterialManager", "load_scene_file"]
