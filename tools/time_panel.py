#!/usr/bin/env python3
"""Phase split of the multi-workgroup band reduction's panel kernel (s_memtime cycles, summed
over the 32 panels of one n = 513 cell), 14 cells per launch (the 8-GPU shard size)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PFML_BAND_MODE"] = "multi"
from pfml.ops import _native as nat  # noqa: E402
from tools.bench_band import run  # noqa: E402

ncells = int(sys.argv[1]) if len(sys.argv) > 1 else 14
dev = torch.device("cuda", 0)
run(ncells, 513, reps=1)
buf = torch.zeros(ncells * 8 + 16, dtype=torch.int64, device=dev)
nat.hip_lib().pfml_ridge_set_timing(buf.data_ptr())
run(ncells, 513, reps=1)          # warm-up launch + 1 rep: 2 accumulations
torch.cuda.synchronize()
nat.hip_lib().pfml_ridge_set_timing(None)
t = buf.cpu().numpy()[: ncells * 8].reshape(ncells, 8)[:, :5].mean(0) / 2.0
names = ["load", "qr", "G_T", "U_V_store", "-"]
tot = t.sum()
print(json.dumps({nm: f"{v:.0f} cyc ({100 * v / tot:.1f}%), {v / 32:.0f}/panel"
                  for nm, v in zip(names, t)}))
