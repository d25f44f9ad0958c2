"""The CPU oracle (the parity checker) under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5): every entry point on a scene with triangles, a rect and spheres. Host code only —
GPU sanitizers are not available on the MI355X pool."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_sanitized")
    build = subprocess.run(
        ["gcc", "-O1", "-g", "-std=c11", "-fno-omit-frame-pointer", "-ffp-contract=off", "-fno-fast-math",
         "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
         os.path.join(ORACLE, "mfx_oracle.c"), os.path.join(ORACLE, "sanitize_driver.c"), "-lm", "-o", exe],
        capture_output=True, text=True)
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert run.returncode == 0, (run.returncode, run.stdout[-2000:], run.stderr[-4000:])
    assert "runtime error" not in run.stderr and "ERROR: AddressSanitizer" not in run.stderr, run.stderr[-4000:]
    assert "rays hit" in run.stdout
