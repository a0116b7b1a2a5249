"""The programs under examples/ run: the PyTorch ones here on the CPU (the
row-split one as two gloo ranks), the C one built against the headers and the
in-tree library."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, **kw):
    env = dict(os.environ, VELES_DISABLE_GPU="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600, **kw)
    assert r.returncode == 0, r.stdout[-1500:] + r.stderr[-1500:]
    return r.stdout


def test_wavelet_features_example():
    out = _run([sys.executable, "examples/wavelet_features.py"])
    assert "step 4: loss" in out
    losses = [float(line.split()[-1]) for line in out.splitlines() if line.startswith("step")]
    assert losses[-1] < losses[0]


def test_rowsplit_example_two_gloo_ranks():
    out = _run([sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr",
                "127.0.0.1", "--nproc-per-node", "2", "examples/rowsplit_torchrun.py"])
    assert "world 2" in out


def test_convolve_demo_builds_and_runs(tmp_path):
    from veles.simd_amd import _lib
    exe = str(tmp_path / "convolve_demo")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-O1", "examples/convolve_demo.c", "-Iinclude", "-L" + libdir,
                    "-lvelessimd", "-lm", "-Wl,-rpath," + libdir, "-o", exe],
                   cwd=REPO, check=True, capture_output=True)
    out = _run([exe])
    assert "overlap-save" in out
