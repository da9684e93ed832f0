#!/usr/bin/env python3
"""% of peak of the headline grid step's kernels, from a kernel timeline
(tools/rocprof_timeline.py output of one `bench.py --no-inputs` step).

Ceilings measured on MI355X (profiles/r03_mfma_f64_peak_v2.json): fp64 MFMA 78.2 TF/s
(64 cycles per v_mfma_f64_16x16x4 per SIMD, 1024 SIMDs, 2.39 GHz; spec 78.6), fp64 VALU FMA
65.7 TF/s; HBM3E 8 TB/s (spec).  Flop / byte counts are the work each kernel executes for the
headline config (2 g x 53 years, n = 513 / 257 / 129 / 65, 101 lambdas, 12 validation months,
710 months of 513 x 513 summands); the 106 big cells' reduction runs on 106 of 256 CUs, so
its per-CU efficiency is quoted too.  (The reduction kernel is band_coop_kernel; its two
launches - the big cells' and the rest - are told apart by their queues.)

usage: python tools/roofline.py profiles/r04_step_timeline.txt > profiles/r04_roofline_grid_step.md
"""
import re
import sys

MFMA, VALU, HBM = 78.2e12, 65.7e12, 8.0e12
G, Y, L, NV = 2, 53, 101, 12
BIG, SMALL = [513], [257, 129, 65]


def cells(ns):
    return G * Y * len(ns), ns


def red_flops(ns):                      # two-sided band reduction: 4/3 n^3 per cell
    return sum(G * Y * 4.0 / 3.0 * n ** 3 for n in ns)


def solve_flops(ns):                    # banded Cholesky + 2 triangular solves, b = 16, per lambda
    return sum(G * Y * L * n * (2 * 16 * 17 + 4 * 16) for n in ns)


def bt_flops(ns):                       # blocked-WY back-transform: 4 n^2 per lambda (V'Y, V M)
    return sum(G * Y * L * 4.0 * n * n for n in ns)


def quad_flops(ns):                     # upper block triangle, 64-row tiles, 112 padded lambdas
    tot = 0.0                           # (the tail index of n = 64k + 1 is off the tiles)
    for n in ns:
        nm = n - 1 if (n > 1 and (n - 1) % 16 == 0) else n
        nt = (nm + 63) // 64
        k = sum(nm - 64 * i for i in range(nt))
        tot += G * Y * NV * 2.0 * 64 * 112 * k
    return tot


def main():
    rows = []
    for line in open(sys.argv[1]):
        m = re.match(r"\s*(\S.*?)\s+(\d+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s*$", line)
        if m:
            rows.append((m.group(1).strip(), int(m.group(2)), float(m.group(3)),
                         float(m.group(4)), float(m.group(5))))
    # the last full step: from the last wsum_upper to the last dense_rank
    i0 = max(i for i, r in enumerate(rows) if r[0].startswith("wsum_upper"))
    step = rows[i0:]
    i1 = max(i for i, r in enumerate(step) if r[0].startswith("dense_rank"))
    step = step[:i1 + 1]
    t0, t1 = step[0][2], step[-1][3]
    by = {}
    for name, q, a, b, d in step:
        key = name.split("<")[0].split("(")[0]
        if key.startswith("band_coop_kernel"):
            key = "ridge_band_reduce_kernel"
        by.setdefault(key, []).append((q, d))
    red = by.get("ridge_band_reduce_kernel", [])
    big_q = max(red, key=lambda x: x[1])[0] if red else None   # the big cells' queue
    def dur(key, big):
        ds = [(q, d) for q, d in by.get(key, [])]
        if not ds:
            return None
        if len(ds) == 1:
            return ds[0][1]
        pick = [d for q, d in ds if (q == big_q) == big]
        return pick[0] if pick else None
    P, T = 513, 710
    wsum_bytes = G * T * P * (P + 1) / 2 * 8
    table = [
        ("wsum_upper_kernel (window segment sums)", dur("wsum_upper_kernel", True), None, wsum_bytes, "HBM"),
        ("wsum_chunk_totals + prefix (windows)", (dur("wsum_chunk_totals_kernel", True) or 0) + (dur("wsum_chunk_prefix_kernel", True) or 0), None,
         G * 61 * P * (P + 1) / 2 * 8 * 2 + G * Y * P * P * 8, "HBM"),
        ("band reduction, 106 n=513 cells", dur("ridge_band_reduce_kernel", True), red_flops(BIG), None, "MFMA"),
        ("band reduction, 318 small cells", dur("ridge_band_reduce_kernel", False), red_flops(SMALL), None, "MFMA"),
        ("banded Cholesky solves, big", dur("ridge_band_solve_kernel", True), solve_flops(BIG), None, "VALU"),
        ("banded Cholesky solves, small", dur("ridge_band_solve_kernel", False), solve_flops(SMALL), None, "VALU"),
        ("back-transform beta = Q y, big", dur("ridge_band_backtransform_kernel", True), bt_flops(BIG), None, "MFMA"),
        ("back-transform beta = Q y, small", dur("ridge_band_backtransform_kernel", False), bt_flops(SMALL), None, "MFMA"),
        ("validation utilities (quadform), big", dur("quadform_kernel", True), quad_flops(BIG), None, "MFMA"),
        ("validation utilities (quadform), small", dur("quadform_kernel", False), quad_flops(SMALL), None, "MFMA"),
    ]
    print(f"# Headline grid step: % of peak per kernel ({sys.argv[1]})\n")
    print(f"step wall time (first to last kernel): {(t1 - t0) / 1e3:.3f} ms\n")
    print("| kernel | us | work | achieved | % of chip peak | note |")
    print("|---|---|---|---|---|---|")
    for name, us, fl, by_, unit in table:
        if not us:
            continue
        if fl is not None:
            rate = fl / (us * 1e-6)
            peak = MFMA if unit == "MFMA" else VALU
            note = ""
            if "106 n=513" in name:
                note = f"{100 * rate / (peak * 106 / 256):.1f} % of the 106 CUs it runs on"
            print(f"| {name} | {us:.0f} | {fl / 1e9:.1f} GFLOP | {rate / 1e12:.1f} TF/s | "
                  f"{100 * rate / peak:.1f} % ({unit} {peak / 1e12:.1f}) | {note} |")
        else:
            rate = by_ / (us * 1e-6)
            print(f"| {name} | {us:.0f} | {by_ / 1e9:.2f} GB | {rate / 1e12:.2f} TB/s | "
                  f"{100 * rate / HBM:.1f} % (HBM 8 TB/s) | |")


if __name__ == "__main__":
    main()
