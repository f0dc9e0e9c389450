"""Drive scripts/dma_slot_race.hip (build: see its header): stale reads of per-wave LDS-DMA slots, per variant and
wave, over repeated launches.
  variant 0: no stagger, slot read after quadrant 2 by column waves 0/1     (the product GEMM's order, LDS form)
  variant 1: wave row 1 issues its pieces after quadrant 1 (stagger), same reads
  variant 2: stagger, every slot read after quadrant 4
  variant 3: stagger, slots below the ring (offset 0) instead of at 138 KiB
  variant 4: as 1 with transposed (ds_read_b64_tr_b16) operand reads; variant 5: as 4 without the stagger
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, 'scripts', 'libdmarace.so'))
lib.dma_race_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device('cuda', 0)
ntiles = 512
w = torch.arange(ntiles * 64, device=dev, dtype=torch.float32)
src_pieces = 8192
src = torch.randn(src_pieces * 512, device=dev).bfloat16()
sink = torch.zeros(512, device=dev)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for nblocks in (32, 256):
    for variant in (0, 1, 2, 3, 4, 5):
        bad = torch.zeros(8, device=dev, dtype=torch.int32)
        runs_bad = 0
        for _ in range(reps):
            before = bad.clone()
            rc = lib.dma_race_run(variant, w.data_ptr(), src.data_ptr(), src_pieces, ntiles, nblocks, bad.data_ptr(),
                                  sink.data_ptr(), torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
            torch.cuda.synchronize()
            runs_bad += int((bad - before).sum().item() > 0)
        print(f'blocks {nblocks:3d} variant {variant}: {runs_bad:2d}/{reps} runs with stale slot values; '
              f'per wave (w0..w7 = wr0 wc0-3, wr1 wc0-3): {bad.tolist()}', flush=True)
