"""Step-by-step lockstep run on the known-answer graph with synchronisation and dumps."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sheep_amd import device  # noqa: E402
from sheep_amd.dist import shard_bounds  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 3
device.init(0)
ka = np.array([[0, 1], [1, 0], [2, 2], [1, 2], [3, 4], [4, 1], [6, 5], [5, 6], [5, 6], [2, 4]],
              np.uint32)
full = torch.from_numpy(ka.view(np.int32)).cuda().view(torch.uint32)
shards = [full[slice(*shard_bounds(10, r, P))].contiguous() for r in range(P)]
parts = [device.degree_ex(uv, 7, 0) for uv in shards]
deg = parts[0][0].clone()
for d, _ in parts[1:]:
    deg.view(torch.int32).add_(d.view(torch.int32))
seq, rmap, n_seq = device.sequence(deg)
print("seq", seq[:n_seq].cpu().tolist(), flush=True)
sess = [device.Lockstep(uv, rmap, seq, n_seq, deg) for uv in shards]
torch.cuda.synchronize()
print("bin counts", [s.bin_counts.tolist() for s in sess], flush=True)
g = np.sum([s.bin_counts for s in sess], axis=0)
plans = [s.plan(g) for s in sess]
print("plans", plans, flush=True)
nbk, slots = plans[0]
sends = [torch.zeros(slots + max(uv.shape[0], 1), dtype=torch.int64, device="cuda") for uv in shards]
for k in range(nbk):
    ns = [s.map(k, sends[r]) for r, s in enumerate(sess)]
    torch.cuda.synchronize()
    print("bucket", k, "kept", ns, flush=True)
    cap = max(ns)
    for r, s in enumerate(sess):
        s.pack(k, sends[r], cap)
    torch.cuda.synchronize()
    recv = torch.cat([x[:slots + cap] for x in sends])
    print("recv", [hex(v & (2 ** 64 - 1)) for v in recv.cpu().tolist()], flush=True)
    for r, s in enumerate(sess):
        s.apply(k, recv, P, cap)
        torch.cuda.synchronize()
        print("applied", r, flush=True)
for r, s in enumerate(sess):
    p, w = s.finish(seq, parts[r][0], parts[r][1], 0)
    print("rank", r, p[:n_seq].cpu().numpy().view(np.uint32).tolist(),
          w[:n_seq].cpu().numpy().view(np.uint32).tolist(), flush=True)
