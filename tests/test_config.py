"""The knob registry (veles/simd_amd/utils/config.py) lists every
environment variable the native sources and the Python layer read, and the
profiling ranges are wired into the native-call path."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env_reads():
    names = set()
    pat = re.compile(r'(?:getenv|env_int)\("((?:VELES|VS)_[A-Z0-9_]+)"')
    for d, _, files in os.walk(os.path.join(ROOT, "csrc")):
        for f in files:
            if f.endswith((".cpp", ".h", ".hip")):
                names |= set(pat.findall(open(os.path.join(d, f)).read()))
    pat_py = re.compile(r'environ\.get\("((?:VELES|VS)_[A-Z0-9_]+)"')
    for f in ("_lib.py",):
        names |= set(pat_py.findall(open(os.path.join(ROOT, "veles", "simd_amd", f)).read()))
    return names


def test_every_env_knob_is_registered():
    from veles.simd_amd.utils import BY_NAME
    reads = _env_reads()
    assert reads, "regex found nothing"
    missing = sorted(reads - set(BY_NAME))
    assert not missing, f"env knobs read but not documented in utils/config.py: {missing}"
    stale = sorted(n for n in BY_NAME if n not in reads)
    assert not stale, f"documented knobs nobody reads: {stale}"


def test_describe_prints_table():
    out = subprocess.run([sys.executable, "-m", "veles.simd_amd.utils.config"], cwd=ROOT,
                         capture_output=True, text=True, check=True,
                         env=dict(os.environ, VELES_LOG_LEVEL="2")).stdout
    assert "| `VELES_LOG_LEVEL` | 2 |" in out


def test_profile_ranges_wrap_native_calls():
    """VELES_PROFILE_RANGES=1: _lib.call pushes / pops one range per call."""
    code = (
        "import veles.simd_amd._lib as L, veles.simd_amd.utils.profiling as P\n"
        "seen = []\n"
        "P._ENABLED = True\n"
        "import torch\n"
        "torch.cuda.is_available = lambda: True\n"
        "torch.cuda.nvtx.range_push = lambda n: seen.append(('push', n))\n"
        "torch.cuda.nvtx.range_pop = lambda: seen.append(('pop',))\n"
        # a call whose result is 0 with or without a GPU (vs_gpu_available
        # returns 1 on a GPU box, which call() would read as a failed status)
        "L.call('vs_is_device_pointer', None)\n"
        "assert seen == [('push', 'vs_is_device_pointer'), ('pop',)], seen\n"
        "print('ok')\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True,
                         text=True, env=dict(os.environ, VELES_PROFILE_RANGES="1"))
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-2000:]
