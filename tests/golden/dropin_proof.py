#!/usr/bin/env python3
"""Drop-in proof: the reference's own driver runs unchanged on this repository's module.

Runs in the build container only (the GPU box has no /root/reference).  It repeats every case
of make_golden.py -- the reference's unmodified ``ClassLassoCPU`` (lasso.py:25-169), its
``multiprocessing.Pool`` and all -- but with ``sys.modules["cpu_calculation"]`` bound to
``convex_optimization_amd.cpu_calculation`` before the reference's lasso.py is imported, so
lasso.py:17-18 (``from cpu_calculation import element_proj, soft_thresholding, error_crit,
fun_s12, fun_s22, fun_dd_p``) and the harness's ``A_bp_get`` / ``fun_diag_ATA`` all resolve to
the drop-in.  The fixtures go to tests/golden/dropin/; tests/test_oracle.py checks that every
array in them equals the corresponding reference-run fixture (tests/golden/*.npz) bit for bit.

Usage:  python tests/golden/dropin_proof.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import make_golden  # noqa: E402
from convex_optimization_amd import cpu_calculation as dropin  # noqa: E402


def main():
    sys.modules["cpu_calculation"] = dropin          # before the reference's lasso.py is imported
    cc, parameters, lasso = make_golden._import_reference()
    assert cc is dropin and lasso.soft_thresholding is dropin.soft_thresholding
    assert lasso.fun_s12 is dropin.fun_s12 and lasso.fun_s22 is dropin.fun_s22
    out = os.path.join(HERE, "dropin")
    os.makedirs(out, exist_ok=True)
    make_golden.OUT = out
    mods = (dropin, parameters, lasso)
    make_golden.make_case(mods, "c1_b1_p1_f64", 20190325, 512, 2048, 0.4, 1, 1, 200, False)
    make_golden.make_case(mods, "c1_b2_p4_f64", 20190325, 512, 2048, 0.4, 2, 4, 200, False)
    make_golden.make_case(mods, "c1_b1_p1_f32in", 20190326, 512, 2048, 0.4, 1, 1, 200, True)
    make_golden.make_case(mods, "c1_b2_p4_f32in", 20190326, 512, 2048, 0.4, 2, 4, 200, True)
    make_golden.make_case(mods, "ragged_b3_p2_f32in", 4242, 77, 120, 0.4, 3, 2, 60, True)
    make_golden.make_case(mods, "bound_b4_p2_f32in", 99, 96, 320, 0.3, 4, 2, 2000, True, err_bound=1e-3)
    make_golden.make_case(mods, "random_b4_p1_f32in", 1234, 128, 512, 0.4, 4, 1, 64, True,
                          random_order=True, py_seed=5)
    for name, (P, eb) in make_golden.STOP_CASES.items():    # round 6: the one-pass stop rule's pins
        make_golden.make_case(mods, name, 20190327, 256, 4096, 0.4, 1, P, 600, True, err_bound=eb)
    make_golden.make_case(mods, "raggedbound74_b3_p2_f32in", 4242, 77, 120, 0.4, 3, 2, 200, True, err_bound=8.909e-05)
    make_golden.make_case(mods, "randbound231_b4_p2_f32in", 1234, 128, 512, 0.4, 4, 2, 600, True,
                          err_bound=2.5544e-4, random_order=True, py_seed=7)
    make_golden.make_case(mods, "randbound545_b4_p1_f32in", 1234, 128, 512, 0.4, 4, 1, 800, True,
                          err_bound=7.16e-6, random_order=True, py_seed=7)
    bad = []
    for name in sorted(os.listdir(out)):
        a = np.load(os.path.join(out, name))
        b = np.load(os.path.join(HERE, name))
        for k in b.files:
            if not np.array_equal(a[k], b[k]):
                bad.append((name, k))
    print("drop-in fixtures equal to the reference-run fixtures bit for bit:", not bad, bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
