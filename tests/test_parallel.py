"""Multi-process tests of the parallel layer: gloo backend on CPU, world
size 2 (and 3 for uneven shards), rendezvous on 127.0.0.1."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, fn, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in results if isinstance(r, str)]
    assert not errs, errs[0]
    return sorted(results)


def _worker(rank, world, port, fn, args, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        from veles.simd_amd import parallel
        parallel.init(backend="gloo")
        fn(rank, world, *args)
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put(traceback.format_exc())


def _dp_case(rank, world):
    from veles.simd_amd import ops, parallel
    g = torch.Generator().manual_seed(0)
    x = torch.randn(7, 300, generator=g)
    h = torch.randn(20, generator=g)
    y = parallel.dp_apply(ops.conv1d, x, h)
    torch.testing.assert_close(y, ops.conv1d(x, h))
    part = parallel.dp_apply(ops.conv1d, x, h, gather=False)
    a, b = parallel.shard_range(7, world, rank)
    torch.testing.assert_close(part, ops.conv1d(x[a:b], h))


def _rowsplit_case(rank, world):
    from veles.simd_amd import parallel
    g = torch.Generator().manual_seed(1)
    a = torch.randn(3, 8 * world, 16, generator=g)
    b = torch.randn(3, 16, 12, generator=g)
    m = a.shape[1] // world
    c = parallel.rowsplit_bmm(a[:, rank * m:(rank + 1) * m].contiguous(), b)
    torch.testing.assert_close(c, torch.bmm(a, b), atol=1e-4, rtol=1e-4)
    c2 = parallel.rowsplit_bmm(a[:, rank * m:(rank + 1) * m].contiguous(),
                               b if rank == 0 else None, n=12, broadcast_src=0)
    torch.testing.assert_close(c2, torch.bmm(a, b), atol=1e-4, rtol=1e-4)


def _cp_conv_case(rank, world, corr):
    from veles.simd_amd import ops, parallel
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 1000, generator=g)
    h = torch.randn(37, generator=g)
    a, b = parallel.shard_range(1000, world, rank)
    y = parallel.cp_conv1d(x[:, a:b].contiguous(), h, correlate=corr)
    full = ops.conv1d(x, h, correlate=corr)
    stop = full.shape[-1] if rank == world - 1 else b
    torch.testing.assert_close(y, full[:, a:stop], atol=1e-4, rtol=1e-4)


def _cp_swt_case(rank, world, ext):
    from veles.simd_amd import ops, parallel
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 512, generator=g)
    a, b = parallel.shard_range(512, world, rank)
    hi, lo = parallel.cp_swt(x[:, a:b].contiguous(), "db", 8, levels=3, ext=ext)
    fhi, flo = ops.swt(x, "db", 8, levels=3, ext=ext)
    torch.testing.assert_close(hi, fhi[..., a:b], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(lo, flo[..., a:b], atol=1e-4, rtol=1e-4)


def test_data_parallel_world2():
    _run(2, _dp_case)


def test_data_parallel_uneven_world3():
    _run(3, _dp_case)


def test_rowsplit_bmm_world2():
    _run(2, _rowsplit_case)


@pytest.mark.parametrize("corr", [False, True])
def test_context_parallel_conv_world2(corr):
    _run(2, _cp_conv_case, corr)


@pytest.mark.parametrize("ext", ["periodic", "mirror", "constant", "zero"])
def test_context_parallel_swt_world2(ext):
    _run(2, _cp_swt_case, ext)


def test_shard_range():
    from veles.simd_amd.parallel import shard_range
    assert [shard_range(10, 3, r) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert shard_range(5, 1, 0) == (0, 5)
