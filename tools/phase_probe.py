"""Development probe: per-phase timing of the Cholesky kernels from s_memtime stamps.
Run with the phase build:  make -C g2o_amd phases && G2OHIP_LIB=g2o_amd/libg2o_hip_phases.so python tools/phase_probe.py
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import g2o_amd  # noqa: E402
from g2o_amd import synth  # noqa: E402

CLK = 2.4e3  # s_memtime ticks per microsecond (core clock counter)


def main():
    prob = synth.by_name(sys.argv[1] if len(sys.argv) > 1 else "C4")
    opt = g2o_amd.SparseOptimizer(0).add_problem(prob)
    L = g2o_amd.lib()
    opt.optimize_step(0)
    buf = (C.c_ulonglong * (8 * 4096))()
    L.g2ohip_debug_phases(buf, 4096)  # drop warmup records
    opt.optimize_step(1)
    n = L.g2ohip_debug_phases(buf, 4096)
    a = np.frombuffer(buf, dtype=np.uint64, count=8 * n).reshape(n, 8).astype(np.int64)
    print(f"{n} records")
    periods(a)
    tail(a)
    for kid, name, labels in ((1, "k_extend_add block-0 task", ["stage+assemble", "factor", "publish"]),
                              (2, "k_step(diag task)", ["stage+trsm+syrk", "factor", "publish"]),
                              (3, "k_step(tile 0,0)", ["stage", "trsm+L21", "update+store"])):
        r = a[a[:, 0] == kid]
        if len(r):
            d = r[:, 6] - r[:, 5]
            ok = (r[:, 6] > 0) & (r[:, 5] > 0)
            if ok.any():
                print(f"{name}: chol32 alone median {np.median(d[ok]) / CLK:7.2f} us  (n={ok.sum()})")
        r = a[a[:, 0] == kid]
        if not len(r):
            continue
        print(f"{name}: {len(r)} launches")
        t = r[:, 1:]
        for i, lab in enumerate(labels):
            d = t[:, i + 1] - t[:, i]
            ok = (t[:, i + 1] > 0) & (t[:, i] > 0)
            if ok.any():
                print(f"   {lab:16s} median {np.median(d[ok]) / CLK:7.2f} us  mean {np.mean(d[ok]) / CLK:7.2f} us  (n={ok.sum()})")


def tail(a):
    """Per k_step launch: start of the last-dispatched workgroup and its end, relative to the diagonal task's start."""
    ids = a[:, 0]
    rs, re_, span = [], [], []
    for k in range(1, len(a)):
        if ids[k] == 3 and ids[k - 1] == 2 and a[k, 7] > 0:  # s_memrealtime (100 MHz, chip-wide) stamps
            rs.append((a[k, 6] - a[k - 1, 7]) / 100.0)
            re_.append((a[k, 7] - a[k - 1, 7]) / 100.0)
            span.append((a[k - 1, 4] - a[k - 1, 1]) / CLK)
    if rs:
        print(f"last workgroup vs diagonal task (n={len(rs)}): start +{np.median(rs):.2f} us, end +{np.median(re_):.2f} us "
              f"(max {np.max(re_):.2f}), diagonal task span {np.median(span):.2f} us")
    r = a[ids == 2]
    for q in range(min(len(r), 60)):
        t = r[q]
        print(f"   diag {q:3d}: stage {(t[2] - t[1]) / CLK:5.2f}  pre-chol {(t[5] - t[2]) / CLK:5.2f}  chol32 {(t[6] - t[5]) / CLK:5.2f}"
              f"  post {(t[3] - t[6]) / CLK:5.2f}" + (f"  | last end +{re_[q]:5.2f}" if q < len(re_) else ""))


def periods(a):
    """Diag-task chain: start-to-start period of consecutive k_step diag records vs the task's own span."""
    r = a[a[:, 0] == 2]
    if len(r) < 3:
        return
    st = r[:, 1]
    en = r[:, 4]
    per = np.diff(st) / CLK
    own = (en - st) / CLK
    ok = (per > 0) & (per < 100)
    print(f"diag chain: period median {np.median(per[ok]):.2f} us, task span median {np.median(own):.2f} us, "
          f"gap (period - span) median {np.median(per[ok] - own[:-1][ok]):.2f} us")


if __name__ == "__main__":
    main()
