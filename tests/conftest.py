import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SCENES = os.path.join(ROOT, "scenes")
SEED = 0x4D414652


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmafrix_rt.so on the GPU)")


def gpu_available() -> bool:
    try:
        from mafrixraytracing_amd.abi import load_library
        return load_library().mfx_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def gpu():
    from mafrixraytracing_amd.abi import load_library
    lib = load_library()  # fails loudly if the HIP build is missing
    if lib.mfx_device_count() < 1:
        pytest.fail("no HIP device visible (gpu tests must run on the MI355X box)")
    return lib


def scene(name, w=None, h=None, max_depth=3):
    """scenes/<name>.xml; "<name>@2l": an instanced scene traced two-level (MFX_F_TWO_LEVEL) instead
    of the library's default (flattened when it fits)."""
    from mafrixraytracing_amd.scene_io import load_scene_file
    two = name.endswith("@2l")
    a = load_scene_file(os.path.join(SCENES, name.replace("@2l", "") + ".xml"), max_depth=max_depth)
    a.two_level = two
    if w is not None:
        a = a.with_film(w, h)
    return a
