"""Runs the native C API test binary (source-compatibility + goldens)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "tests", "capi_test")


def _run(extra_env):
    if not os.path.exists(BIN):
        from veles.simd_amd import build
        build.build()
    env = dict(os.environ, **extra_env)
    res = subprocess.run([BIN], capture_output=True, text=True, env=env,
                         timeout=600)
    assert res.returncode == 0, res.stdout + res.stderr


def test_native_capi_host():
    _run({"VELES_DISABLE_GPU": "1"})


@pytest.mark.gpu
def test_native_capi_gpu():
    _run({})
