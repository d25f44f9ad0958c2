"""The per-lane kernels' FP16 nodes (MfxNodeH, mfx_layout.h; VERDICT r05 Next #4b): each child box is
the FP32 one rounded outward, so a lane walks a superset of its FP32 walk and the leaf tests decide the
hits. Images and ray counts must equal the FP32-node walk's (MFX_NODE_F32=1, the same library) and the
oracle's bit for bit: flat scenes with the ray queues on and off, a two-level instanced scene, and a
sphere scene."""
import numpy as np
import pytest

from conftest import SEED, scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,w,h,spp", [("spot", 64, 36, 6), ("renault", 40, 24, 4), ("cube_cornell", 48, 27, 5),
                                          ("two_spheres_plane", 32, 32, 4), ("spot16_instanced@2l", 40, 24, 3)])
@pytest.mark.parametrize("queue_from", ["-2", "-1"])
def test_fp16_nodes_equal_fp32_nodes_and_oracle(gpu, oracle, monkeypatch, name, w, h, spp, queue_from):
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, w, h)
    monkeypatch.setenv("MFX_QUEUE_FROM", queue_from)
    monkeypatch.setenv("MFX_CAMERA_PACKETS", "0")  # every camera ray through k_extend's per-lane walk too
    with NativeContext(a, seed=SEED) as c:
        f16 = c.sample(spp)
        n16 = c.ray_counts()[:4]
    monkeypatch.setenv("MFX_NODE_F32", "1")
    with NativeContext(a, seed=SEED) as c:
        f32 = c.sample(spp)
        n32 = c.ray_counts()[:4]
    assert np.array_equal(f16, f32)
    assert np.array_equal(n16, n32)
    assert np.array_equal(f16, oracle.OracleScene(a).sample(spp, SEED, sample_base=0))
