"""The host C API called from several host threads at once (ctypes releases the
GIL for the duration of a call): every thread has its own staging arena, scratch
vectors and error slot, the device work shares the library stream.  Runs on the
host paths without a GPU and through the GPU paths on a GPU box (the larger
shapes below are past every small-call limit).  The reference is reentrant by
construction (pure functions over caller memory, /root/reference/src/convolve.c:49-100)."""
import threading

import numpy as np
import pytest

from veles.simd_amd import capi


def _work(seed, rounds, errors):
    try:
        rng = np.random.default_rng(seed)
        x = rng.standard_normal(3000 + 17 * seed).astype(np.float32)
        h = rng.standard_normal(90 + seed).astype(np.float32)
        xl = rng.standard_normal(40000 + 1001 * seed).astype(np.float32)
        hl = rng.standard_normal(700 + 3 * seed).astype(np.float32)
        a = rng.uniform(-1, 1, (64 + seed, 96)).astype(np.float32)
        b = rng.uniform(-1, 1, (96, 80 + seed)).astype(np.float32)
        big = rng.uniform(-1, 1, (200, 300)).astype(np.float32)
        v = rng.uniform(0.1, 5.0, 5000 + seed).astype(np.float32)
        sig = rng.standard_normal(30000 + seed).astype(np.float32)
        src = rng.standard_normal(512).astype(np.float32)
        want = {
            "conv": np.convolve(x.astype(np.float64), h.astype(np.float64)),
            "convl": np.convolve(xl.astype(np.float64), hl.astype(np.float64)),
            "mm": a.astype(np.float64) @ b.astype(np.float64),
            "add": (big + big).ravel(),
            "exp": np.exp(v.astype(np.float64)),
            "peaks": capi.detect_peaks(0, sig, 3),
            "dwt": capi.wavelet_apply(0, 8, 0, src, na=True),
        }
        for _ in range(rounds):
            assert np.abs(capi.convolve_simd(1, x, h) - want["conv"]).max() < 2e-3
            assert np.abs(capi.convolve_simd(1, xl, hl) - want["convl"]).max() < 2e-2
            res, _ = capi.run_handle("convolve", xl, hl)
            assert np.abs(res - want["convl"]).max() < 2e-2
            got = capi.matrix_multiply(1, a, b, 96, a.shape[0], b.shape[1], 96)
            assert np.abs(got.reshape(want["mm"].shape) - want["mm"]).max() < 2e-4
            assert np.array_equal(capi.matrix_add(1, big, big, 300, 200), want["add"])
            got = capi.psv("exp_psv", 1, v).astype(np.float64)
            assert (np.abs(got - want["exp"]) <= 4e-7 * want["exp"]).all()
            assert capi.detect_peaks(1, sig, 3) == want["peaks"]
            hi, lo = capi.wavelet_apply(0, 8, 0, src)
            assert np.abs(hi - want["dwt"][0]).max() < 1e-5
            assert np.abs(lo - want["dwt"][1]).max() < 1e-5
    except BaseException as e:  # noqa: BLE001
        errors.append((seed, repr(e)))


def _run(nthreads, rounds):
    errors = []
    threads = [threading.Thread(target=_work, args=(i, rounds, errors)) for i in range(nthreads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "a worker thread did not finish"
    assert not errors, errors


def test_host_api_from_many_threads_host_paths():
    _run(8, 5)


@pytest.mark.gpu
def test_host_api_from_many_threads_gpu_paths():
    _run(8, 10)


def test_native_thread_test_binary():
    """tests/native/threads_test.cpp (the program `make tsan` runs under
    ThreadSanitizer) built against the regular library: 8 threads x 3 rounds."""
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, "build", "tests", "threads_test")
    if not os.path.exists(exe):
        pytest.skip("build/tests/threads_test not built (make tests)")
    r = subprocess.run([exe, "8", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout


@pytest.mark.gpu
def test_short_lived_threads_reuse_staging_images():
    """Threads that end hand their pinned staging image (16 MiB of pinned host
    and of device memory) to the next thread that needs one: thirty threads in
    a row, each making GPU calls on host arrays, hold one image between them."""
    import torch
    rng = np.random.default_rng(3)
    big = rng.uniform(-1, 1, (200, 300)).astype(np.float32)
    errors = []

    def one():
        try:
            assert np.array_equal(capi.matrix_add(1, big, big, 300, 200), (big + big).ravel())
        except BaseException as e:  # noqa: BLE001
            errors.append(repr(e))

    def spawn(n):
        for _ in range(n):
            t = threading.Thread(target=one)
            t.start()
            t.join()

    spawn(2)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    spawn(30)
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert not errors, errors
    assert free0 - free1 < (32 << 20), (free0, free1)   # 30 images would be 480 MiB


@pytest.mark.gpu
def test_long_calls_in_pieces_from_several_threads():
    """Long math calls and long convolutions go through each thread's own staging
    image in overlapped pieces while sharing the library stream: four threads at
    once, every result checked."""
    from scipy.signal import fftconvolve
    errors = []

    def work(seed):
        try:
            rng = np.random.default_rng(100 + seed)
            n = 3 * 262144 + 1000 * seed + 5
            v = rng.uniform(0.1, 6.0, n).astype(np.float32)
            want_log = np.log(v.astype(np.float64))
            x = rng.standard_normal((3 << 19) + 4096 * seed + 9).astype(np.float32)
            h = rng.standard_normal(300 + seed).astype(np.float32)
            want_conv = fftconvolve(x.astype(np.float64), h.astype(np.float64))
            for _ in range(3):
                got = capi.psv("log_psv", 1, v).astype(np.float64)
                assert (np.abs(got - want_log) <= 4e-7 * np.abs(want_log) + 5e-7).all()
                assert np.abs(capi.convolve_simd(1, x, h) - want_conv).max() <= 2e-3
        except BaseException as e:  # noqa: BLE001
            errors.append((seed, repr(e)))

    threads = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
