"""BASELINE.md §3 rows from a tools/sweep.py --vendor run (profiles/<tag>/sweep_all.jsonl).

B_alg = 8(M+1) + 20 nnz(A) + 12 flop + 12 nnz(C); compulsory bytes =
8(M+1) + 12 nnz(A) + 12 nnz(C) (read A once, write C once; A*A reads B = A).
usage: python tools/baseline_table.py profiles/r02h/sweep_all.jsonl"""
import json
import sys

PEAK = 8000.0
print("| Matrix (stand-in) | rows | flop | nnz(C) | t_e2e ms | GFLOPS (t_e2e) | GFLOPS (t_ref) "
      "| B_alg GB/s | % roofline (B_alg) | % roofline (compulsory) | rocSPARSE ms | × rocSPARSE |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|")
for line in open(sys.argv[1]):
    d = json.loads(line)
    M, nA, fl, nC = d["rows"], d["nnzA"], d["flop"], d["nnzC"]
    t = d["total_e2e"]
    tref = t - d["Form_mask_matrix_B"]
    balg = 8 * (M + 1) + 20 * nA + 12 * fl + 12 * nC
    comp = 8 * (M + 1) + 12 * nA + 12 * nC
    gb = balg / (t * 1e-3) / 1e9
    gc = comp / (t * 1e-3) / 1e9
    v = d.get("rocsparse_ms")
    print(f"| {d['matrix']} | {M:,} | {fl:.3g} | {nC:.3g} | {t:.3f} | {2 * fl / (t * 1e-3) / 1e9:.1f} "
          f"| {2 * fl / (tref * 1e-3) / 1e9:.1f} | {gb:.0f} | {100 * gb / PEAK:.1f} | {100 * gc / PEAK:.1f} "
          f"| {v if v is None else f'{v:.3f}'} | {'' if not v else f'{v / t:.2f}'} |")
