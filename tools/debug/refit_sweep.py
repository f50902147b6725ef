"""Sweep of tools/debug/refit_spread.py over the fuzz families (CPU): per method, the worst
difference from skimage in the tests metric and the cases beyond max(1e-8, 100 x LAPACK spread).

    python tools/debug/refit_sweep.py <affine|projective> <n_seeds> <start_seed>
"""
import sys, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
import refit_spread as RS, oracle
model = sys.argv[1]; n = int(sys.argv[2]); start=int(sys.argv[3])
keys = ["scipy gesvd", "r5 GPU: chol inv-iter on AtA", "givens QR + jacobi(R)", "r6 GPU: householder + inv-iter / jacobi", "lapack spread"]
rows = []
for seed in range(start, start+n):
    for f in range(12):
        src, dst = RS.case(seed, f, model)
        if len(src) < 3: continue
        H, inl, bt, ni = oracle.ransac_model(src, dst, model)
        ms = 3 if model=="affine" else 4
        if ni < ms or np.isnan(H).any(): continue
        try:
            o = RS.spread(src, dst, model, verbose=False)
        except (ZeroDivisionError, np.linalg.LinAlgError): continue
        rows.append((seed, f, o))
print(model, "cases", len(rows))
for lim in [1e-10, 1e-8, 1e-6, 1e-4, np.inf]:
    sel = [r for r in rows if r[2]["lapack spread"] <= lim]
    line = f" spread<={lim:g}: n={len(sel)}"
    for k in keys[:-1]:
        w = max([r[2][k] for r in sel], default=0)
        ratio = max([r[2][k] / max(r[2]["lapack spread"], 1e-16) for r in sel], default=0)
        nb = sum(r[2][k] > max(1e-8, 100 * r[2]["lapack spread"]) for r in sel)
        line += f"\n    {k:34s} worst {w:.2g}  worst/spread {ratio:.2g}  n>max(1e-8,100*spread) {nb}"
    print(line)
