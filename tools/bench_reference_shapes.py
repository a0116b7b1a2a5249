#!/usr/bin/env python3
"""Reference benchmark shapes, reference CPU code vs this library, same host.

  python tools/bench_reference_shapes.py build   # here: compiles both drivers
  python tools/bench_reference_shapes.py run     # GPU box: runs both, writes JSON

`build` compiles bench/ref_shapes.cc (1) against the reference sources in
/root/reference (-O2 -march=native, its documented flags, common.ac:267; the
external FFTF library is unavailable offline, so its FFT / overlap-save rows
are compiled out: parity unpinned) into build/bench/ref_shapes_reference, and
(2) against libvelessimd.so (with the device-resident rows) into
build/bench/ref_shapes_veles.  Both binaries travel to the GPU box with the
repo snapshot (build/ is git-ignored, not gpurun-ignored), so `run` times the
reference's AVX code and this library on the same machine.  Output:
profiles/r1/reference_shapes.json (microseconds per call and speed-ups).
"""
import json
import os
import subprocess
import sys

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "build", "bench")
FFTF_STUB = r'''
#pragma once
typedef void *FFTFInstance;
#define FFTF_TYPE_REAL 0
#define FFTF_DIRECTION_FORWARD 0
#define FFTF_DIRECTION_BACKWARD 1
#define FFTF_DIMENSION_1D 1
#define FFTF_NO_OPTIONS 0
static inline void *fftf_init(int a, int b, int c, const int *d, int e, const float *f, float *g) { return 0; }
static inline void *fftf_init_batch(int a, int b, int c, const int *d, int e, int f, const float *const *g, float *const *h) { return 0; }
static inline void fftf_calc(void *p) {}
static inline void fftf_destroy(void *p) {}
'''


def build():
    os.makedirs(OUT, exist_ok=True)
    if os.path.isdir(REF):
        stub = os.path.join(OUT, "stub")
        os.makedirs(os.path.join(stub, "fftf"), exist_ok=True)
        with open(os.path.join(stub, "fftf", "api.h"), "w") as f:
            f.write(FFTF_STUB)
        flags = ["-O2", "-march=native", "-I" + os.path.join(REF, "inc"), "-I" + REF,
                 "-I" + os.path.join(REF, "src"), "-I" + stub]
        objs = []
        for src in ("matrix.c", "memory.c", "convolve.c", "wavelet.c", "daubechies.c",
                    "symlets.c", "coiflets.c"):
            o = os.path.join(OUT, "ref_" + src + ".o")
            subprocess.run(["gcc", "-std=gnu99", "-DNDEBUG", "-c", os.path.join(REF, "src", src),
                            "-o", o] + flags, check=True)
            objs.append(o)
        subprocess.run(["g++", "-O2", "-march=native", "-DNO_FFT",
                        os.path.join(REPO, "bench", "ref_shapes.cc")] + objs + flags
                       + ["-o", os.path.join(OUT, "ref_shapes_reference"), "-lm"], check=True)
    lib = os.path.join(REPO, "veles", "simd_amd", "_native")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-DVELES_DEVICE",
                    "--offload-arch=gfx950", "-x", "hip",
                    "-I" + os.path.join(REPO, "include"),
                    os.path.join(REPO, "bench", "ref_shapes.cc"), "-L" + lib, "-lvelessimd",
                    "-Wl,-rpath," + lib, "-o", os.path.join(OUT, "ref_shapes_veles")], check=True)
    print("built", os.listdir(OUT))


def run():
    res = {}
    for name in ("reference", "veles"):
        exe = os.path.join(OUT, "ref_shapes_" + name)
        if not os.path.exists(exe):
            print("missing", exe)
            continue
        env = dict(os.environ)
        if name == "veles":  # the binary's rpath is this container's path
            env["LD_LIBRARY_PATH"] = os.path.join(REPO, "veles", "simd_amd", "_native")
        out = subprocess.run([exe], check=True, capture_output=True, text=True, env=env,
                             timeout=600)
        res[name] = json.loads(out.stdout.strip().splitlines()[-1])
        print(name, json.dumps(res[name]), flush=True)
    cpu = subprocess.run(["bash", "-c", "grep -m1 'model name' /proc/cpuinfo | cut -d: -f2"],
                         capture_output=True, text=True).stdout.strip()
    speedup = {}
    if "reference" in res and "veles" in res:
        for k, v in res["reference"].items():
            if k in res["veles"] and res["veles"][k] > 0:
                speedup[k] = round(v / res["veles"][k], 2)
    doc = {"unit": "microseconds per call (device rows: per signal / matrix)",
           "host_cpu": cpu, "reference_cpu": res.get("reference"),
           "veles_mi355x": res.get("veles"), "speedup_reference_over_veles": speedup,
           "note": "reference FFT / overlap-save rows need FFTF (not available): "
                   "parity unpinned; host-API rows include H2D/D2H staging."}
    path = os.path.join(REPO, "gpurun_out", "reference_shapes.json")  # copied to profiles/
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(speedup))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1] if len(sys.argv) > 1 else "run"]()
