"""Summarise the per-tile clocks a JY_UJ_PROBE build writes (A/B tool)."""
import sys
import numpy as np

a = np.fromfile(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ujprobe.bin", dtype=np.uint64)
i, calls = 0, []
while i < len(a):
    n = int(a[i + 1]); i += 4
    calls.append(a[i:i + 6 * n].reshape(n, 6).astype(np.int64)); i += 6 * n
for r in calls[-1:]:
    kern = (r[:, 0] >> 56) & 0xff; kind = (r[:, 0] >> 48) & 0xff; t = r[:, 0] & 0xffffffff
    t0 = r[:, 1].min()
    for K in (1, 2, 3, 4, 5):
        m = kern == K
        if not m.any():
            continue
        rr, kk, tt = r[m], kind[m], t[m]
        print(f"U{K}: tiles {m.sum()} span {(rr[:, 3].max() - rr[:, 1].min()) / 100:.1f}us "
              f"start {(rr[:, 1].min() - t0) / 100:.1f}us")
        for kd in np.unique(kk):
            q = kk == kd
            comp = (rr[q, 2] - rr[q, 1]) / 100; lb = (rr[q, 3] - rr[q, 2]) / 100
            extra = ""
            if K == 2 and rr[q, 4].any():
                pre = (rr[q, 4] - rr[q, 1]) / 100; fill = (rr[q, 5] - rr[q, 4]) / 100; items = (rr[q, 2] - rr[q, 5]) / 100
                extra = f" | docs {pre.mean():5.2f} windows {fill.mean():5.2f} items {items.mean():5.2f}"
            print(f"  kind {kd:2d}: n={q.sum():5d} compute mean {comp.mean():6.2f} p99 {np.percentile(comp, 99):6.2f} "
                  f"max {comp.max():6.2f}us | scan mean {lb.mean():6.2f}" + extra)
        o = np.argsort(tt); st = (rr[o, 1] - rr[:, 1].min()) / 100
        print("  ticket start quantiles:", [round(float(st[max(0, int(len(st) * f) - 1)]), 1) for f in (0.1, 0.25, 0.5, 0.75, 1.0)])
