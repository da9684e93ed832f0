#!/usr/bin/env python3
"""Latency anatomy of the one-launch SPD inverse node (csrc/spd_inverse.hip
spd_node_sym_kernel, nn = 128): launch time at a small and the production batch, and - with a
library built with -DPFML_NODE_TIMING (PFML_HIP_LIB) - the shader-clock phase timestamps of
workgroup 0 (A21 staging, the two Gauss-Jordan leaves, the four products, the stores).

    PFML_HIP_LIB=<timing build> python tools/micro/node_timing.py [B ...]
"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pfml.ops._native as nat  # noqa: E402
import pfml.ops.linalg  # noqa: E402,F401  (registers pfml_spd_node_sym)

nat.register_hip("pfml_node_timing", [C.c_void_p])
PHASES = ["stage A21", "GJ X11", "W = X11 A12", "S = A22 - A21 W", "GJ X22", "X22 stores",
          "X12 = -W X22", "D = X12 W'", "X11 -= D stores"]


def main():
    Bs = [int(b) for b in sys.argv[1:]] or [36, 715]
    dev = torch.device("cuda", 0)
    lib = nat.hip_lib()
    out = {}
    for B in Bs:
        g = torch.Generator(device=dev).manual_seed(0)
        X = torch.randn(B, 128, 160, generator=g, dtype=torch.float64, device=dev)
        A = X @ X.transpose(1, 2) / 160 + 0.5 * torch.eye(128, dtype=torch.float64, device=dev)
        A = 0.5 * (A + A.transpose(1, 2))
        st = torch.zeros(B, dtype=torch.int32, device=dev)
        W = A.clone()

        def run():
            nat.check(lib.pfml_spd_node_sym(A.data_ptr(), W.data_ptr(), 128, 128 * 128, B, 0, 128,
                                            st.data_ptr(), nat.stream_of(W)), "node")
        run()
        torch.cuda.synchronize()
        err = float((torch.bmm(W, A) - torch.eye(128, device=dev, dtype=torch.float64)).abs().max())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        ts = (C.c_ulonglong * 16)()
        nat.check(lib.pfml_node_timing(ts), "timing")
        t = list(ts)
        rec = {"B": B, "launch_us": round(us, 1), "max_abs_XA_minus_I": err}
        if t[9]:
            rec["phase_cycles"] = {PHASES[k]: int(t[k + 1] - t[k]) for k in range(9)}
            rec["total_cycles"] = int(t[9] - t[0])
        out[B] = rec
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
