#!/usr/bin/env python3
"""Does a small kernel on one stream wait for the big kernels enqueued earlier on another? Host
order per round: big elementwise kernels (~100k workgroups each) on stream A, then a tiny kernel on
stream B; for pairs of the bench's CU-masked streams and plain torch streams. Run under rocprofv3
--kernel-trace and compare start times (tools/gpu/stream_gate.sh)."""
import pathlib
import sys

import torch

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

pkg = bench._load_pkg()
dev = torch.device("cuda", 0)
x = torch.zeros(1024, device=dev)
big = torch.rand(64 << 20, device=dev)
out = torch.empty_like(big)
created = []
s_fe, s_pll, s_post, s_all = bench.cu_masked_streams(torch, pkg, dev, "64", created)
plain_a, plain_b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
torch.cuda.synchronize()
for name, (a, b) in (("post>fe", (s_post, s_fe)), ("fe>post", (s_fe, s_post)), ("all>fe", (s_all, s_fe)),
                     ("plain", (plain_a, plain_b))):
    torch.cuda.synchronize()
    print(name, flush=True)
    for _ in range(4):
        with torch.cuda.stream(a):
            torch.sin(big, out=out)
            torch.sin(out, out=big)
            torch.sin(big, out=out)
        with torch.cuda.stream(b):
            x.add_(1.0)
    torch.cuda.synchronize()
bench.destroy_masked_streams(torch, pkg, dev, created)
