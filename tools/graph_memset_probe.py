"""Probe: hipMemsetAsync captured into a HIP graph, replayed several times
(round 6: statuses came back as pointer-like garbage from the second replay of
a captured decode on). Prints what each replay leaves in the cleared array."""
import sys, torch
sys.path.insert(0, '.')
import zipora_amd as zr
L = zr.load()
for nbytes in (4, 12, 64, 256, 1024, 4096):
    t = torch.full((max(1, nbytes // 4),), 7, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        L.zr_memset_dev(t.data_ptr(), 0, nbytes, torch.cuda.current_stream().cuda_stream)
    res = []
    for rep in range(4):
        t.fill_(7)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        res.append(sorted(set(t.tolist()))[:3])
    print(nbytes, res, flush=True)
