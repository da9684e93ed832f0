#!/usr/bin/env python3
"""S4 roofline table: achieved TF/s / TB/s and % of the measured fp64 MFMA peak (78.2 TF/s,
profiles/r03_mfma_f64_peak_v2.json) and of HBM3E (8 TB/s) per S4 kernel, from one run's
rocprofv3 kernel trace (rocpd .db) joined with the run's work ledger (PFML_WORK_LEDGER,
pfml/utils/work.py: flops and minimum bytes per kernel name, counted by the host wrappers with
the same dispatch rules as the kernels).

    PFML_S4_STREAMS=1 PFML_WORK_LEDGER=ledger.json rocprofv3 --kernel-trace -d prof -o run -- \\
        python3 bench.py --s4-stress 731 --warmup 0      (ONE eager S4 on one stream: per-kernel
                                                          times do not overlap, the ledger
                                                          counts the same launches)
    python tools/roofline_s4.py prof/.../run_results.db ledger.json > profiles/r05_roofline_s4.md

Ledger keys are full kernel names (``dgemm_kernel<false, false, 64, 64, 2, true>``) or name
prefixes (``standardize`` covers standardize_kernel / standardize_reg_kernel<32>).  Kernels the
ledger does not cover are listed with their time only.
"""
import json
import re
import sqlite3
import sys

MFMA, VALU, HBM = 78.2e12, 65.7e12, 8.0e12
ROLE = {
    "dgemm_glds_kernel<false, false, 128, 64, false, 2, 2, 2>": "Horner steps of (24) (row-scaled, gathered addend, output row scale); SPD-inverse W / X12 and DB products",
    "dgemm_glds_kernel<false, false, 128, 64, true, 2, 2, 2>": "T_0 step of (24) (k-scaled)",
    "dgemm_glds_kernel<false, false, 64, 64, false, 2, 2, 2>": "symmetric-mode products: S = A22 - A21 W, Y M^-1, x^2 + 4x, Sigma",
    "dgemm_glds_kernel<false, true, 64, 64, false, 2, 2, 2>": "symmetric-mode X11 -= X12 W'",
    "dgemm_glds_kernel<true, false, 64, 64, true, 2, 2, 2>": "tc = w omega_chg' Lambda omega_chg (k-scaled, symmetric)",
    "dgemm_glds_kernel<true, false, 64, 64, false, 2, 2, 2>": "risk = gamma omega' Sigma omega (symmetric), X' omega",
    "dgemm_kernel<false, false, 64, 64, 1, false, 16, 2>": "odd-width operands (RFF / 1-column products)",
    "spd_node_sym_kernel": "SPD-inverse nodes of 65..128 rows (two 64-leaf Gauss-Jordan + four MFMA products)",
    "spd_leafinv_kernel": "64 x 64 SPD leaf inverses (register Gauss-Jordan)",
    "mfunc_flat_kernel": "m_func elementwise passes, row stream (exactly symmetric operands)",
    "mfunc_sym_kernel": "m_func elementwise passes, tiled (symmetrising)",
    "db_norm_partial_kernel": "Denman-Beavers scaling norms",
    "standardize": "signal gather + standardise + 1/vol (lags 0, 11, 12) and column statistics (lags 1-10)",
    "lu_update_kernel<32>": "LU solve of [const | Omega] (K7): trailing update",
}


def short(name: str) -> str:
    n = re.sub(r"void |\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*", "", n).strip()


def main():
    db, ledger_path = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels").fetchall()
    trace = {}
    for name, s, e in rows:
        k = short(name)
        t = trace.setdefault(k, [0, 0.0])
        t[0] += 1
        t[1] += (e - s) * 1e-9
    ledger = json.load(open(ledger_path))
    total = sum(v[1] for v in trace.values())
    print("# S4 roofline: achieved rate per kernel vs the MI355X fp64 ceilings\n")
    print(f"Trace: `{db.split('/')[-1]}`, {len(rows)} kernel launches, {total * 1e3:.1f} ms of "
          f"kernel time.  Ceilings: fp64 MFMA {MFMA / 1e12:.1f} TF/s (measured), fp64 VALU "
          f"{VALU / 1e12:.1f} TF/s, HBM3E {HBM / 1e12:.0f} TB/s.  Work per kernel from the run's "
          f"work ledger (`pfml/utils/work.py`).\n")
    print("| kernel | role | launches | ms | GFLOP | TF/s | % fp64 MFMA peak | GB (min) | TB/s "
          "| % HBM |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    used = set()
    out = []
    for key, w in ledger.items():
        names = [k for k in trace if k == key] or [k for k in trace if k.startswith(key)]
        if not names:
            continue
        used.update(names)
        n = sum(trace[k][0] for k in names)
        sec = sum(trace[k][1] for k in names)
        out.append((sec, key, n, w))
    for sec, key, n, w in sorted(out, reverse=True):
        tf = w["flops"] / sec if sec > 0 else 0.0
        bw = w["bytes"] / sec if sec > 0 else 0.0
        calls = f"{n}" if n == w["calls"] else f"{n} (ledger {w['calls']})"
        print(f"| `{key}` | {ROLE.get(key, '')} | {calls} | {sec * 1e3:.1f} | "
              f"{w['flops'] / 1e9:.0f} | {tf / 1e12:.1f} | {100 * tf / MFMA:.0f} % | "
              f"{w['bytes'] / 1e9:.1f} | {bw / 1e12:.2f} | {100 * bw / HBM:.0f} % |")
    rest = sorted(((v[1], k, v[0]) for k, v in trace.items() if k not in used), reverse=True)
    print("\nKernels without a ledger entry (time only):\n")
    print("| kernel | launches | ms |")
    print("|---|---:|---:|")
    for sec, k, n in rest[:15]:
        print(f"| `{k[:90]}` | {n} | {sec * 1e3:.1f} |")
    covered = sum(v[1] for k, v in trace.items() if k in used)
    print(f"\nLedger-covered kernel time: {covered * 1e3:.1f} of {total * 1e3:.1f} ms.")


if __name__ == "__main__":
    main()
