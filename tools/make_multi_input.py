#!/usr/bin/env python3
"""Write NBLOCKS blocks of NCH distinct synthetic channels (bench.make_input, generated on the GPU)
to a file in sdr_multi's input layout ([block][channel][2*block_iq] u8, unpadded rows):
    python tools/make_multi_input.py OUT NCH NBLOCKS"""
from __future__ import annotations

import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def main() -> None:
    out, nch, nblocks = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    import torch
    dev = torch.device("cuda", 0)
    synth = bench._synth_module()
    gen = synth.TorchMultiplexBatch(torch, nch, 0, dev)          # one continuous stream per channel
    buf = torch.empty((nch, 2 * synth.BLOCK_IQ), dtype=torch.uint8, device=dev)
    with open(out, "wb") as f:
        for _ in range(nblocks):
            gen.next_block(out=buf)
            f.write(buf.cpu().numpy().tobytes())
    print(f"{out}: {nch} channels x {nblocks} blocks")


if __name__ == "__main__":
    main()
