import ctypes, sys, torch
sys.path.insert(0, '/root/repo')
from veles.simd_amd import _lib
lib = _lib.lib()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
def run(v, m, n, k, ta, tb, a, b):
    c = torch.full((m, n), 7.0, device='cuda')
    _lib.check(lib.vs_sgemm_variant(v, ta, tb, m, n, k, 1.0, a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1], 0.0, c.data_ptr(), n, s), 'x')
    torch.cuda.synchronize()
    return c
for (m, n, k, ta, tb) in [(128,128,16,0,0),(128,128,16,0,1),(128,128,16,1,0),(128,128,16,1,1),(128,128,64,0,0),(256,256,16,0,0)]:
    for v in (24, 25):
        a = torch.rand((k, m) if ta else (m, k), device='cuda') - 0.5
        b = torch.rand((n, k) if tb else (k, n), device='cuda') - 0.5
        ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
        c = run(v, m, n, k, ta, tb, a, b)
        d = (c.double() - ref).abs()
        bad = (d > 1e-4)
        print(v, (m, n, k, ta, tb), 'maxerr %.3g' % d.max().item(), 'bad frac %.3f' % bad.float().mean().item(),
              'bad rows', bad.any(1).nonzero().flatten()[:8].tolist(), 'bad cols', bad.any(0).nonzero().flatten()[:20].tolist(), flush=True)
