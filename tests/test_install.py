"""`make install` layout + a plain-C consumer linked through the installed
Simd.pc (reference: Simd.pc.in, inc/Makefile.am:27-31, src/Makefile.am:29).

CPU test: installs into a temporary DESTDIR, checks every public header, the
libSimd.so alias and the pkg-config file, then compiles
tests/native/install_consumer.c with gcc using only the .pc's Cflags / Libs
and runs it (host-path calls; no GPU needed)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "veles", "simd_amd", "_native", "libvelessimd.so")


def _pc_fields(path, prefix):
    vars_, fields = {}, {}
    for line in open(path):
        line = line.strip()
        if "=" in line and ":" not in line.split("=")[0]:
            k, v = line.split("=", 1)
            vars_[k] = v
        elif ":" in line:
            k, v = line.split(":", 1)
            fields[k] = v.strip()
    def expand(s):
        for _ in range(3):
            for k, v in vars_.items():
                s = s.replace("${%s}" % k, v)
        return s
    return {k: expand(v) for k, v in fields.items()}


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_install_and_link_c_consumer(tmp_path):
    dest = tmp_path / "stage"
    prefix = "/opt/veles"
    subprocess.run(["make", "-s", "install", f"PREFIX={prefix}", f"DESTDIR={dest}"],
                   cwd=ROOT, check=True, capture_output=True)
    root = dest / prefix.lstrip("/")
    headers = sorted(os.listdir(root / "include" / "simd"))
    assert headers == sorted(os.listdir(os.path.join(ROOT, "include", "simd")))
    for name in ("libvelessimd.so", "libSimd.so", "pkgconfig/Simd.pc"):
        assert (root / "lib" / name).exists(), name
    pc = _pc_fields(root / "lib" / "pkgconfig" / "Simd.pc", prefix)
    assert pc["Name"] == "Simd"
    # the staged tree stands in for the prefix
    cflags = pc["Cflags"].replace(prefix, str(root)).split()
    libs = pc["Libs"].replace(prefix, str(root)).split()
    exe = tmp_path / "consumer"
    subprocess.run(["gcc", "-std=c99", "-O1", *cflags,
                    os.path.join(ROOT, "tests", "native", "install_consumer.c"), "-o", str(exe),
                    *libs, f"-Wl,-rpath,{root / 'lib'}", "-Wl,-rpath,/opt/rocm/lib", "-lm"],
                   check=True)
    env = dict(os.environ, VELES_DISABLE_GPU="1")
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, env=env)
    assert out.stdout.startswith("ok"), out.stdout
