"""TREG LWW at HBM scale, for kernel A/Bs: N keys (default 64M) on one GPU,
batches generated on the device (fresh timestamps 2^18 above the previous
batch in a 2^20 window: ~2/3 of keys win, as bench.py's TREG line; values of
1-8 bytes, so ties are settled by the prefix), the block form
(jy_treg_converge_block) and the keyed form (jy_treg_converge, slot per
entry), each timed by the engine's own HIP events per call.

usage: python tools/treg_hbm.py [KEYS] [STEPS]   (JY_LIB selects a build)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import faulthandler
    faulthandler.dump_traceback_later(float(os.environ.get("JY_DUMP_AFTER", "100")), exit=False)
    import numpy as np
    import torch
    from jylis_amd._lib import TREG
    from jylis_amd.engine import Engine
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda:0")
    eng = Engine(device=0, key_capacity=[1024, 1024, n, 1024, 1024])
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    # fixed-width key strings "t%010d" built on the device, interned there
    idx = torch.arange(n, device=dev, dtype=torch.int64)
    digits = torch.stack([(idx // 10 ** (9 - j)) % 10 + 48 for j in range(10)], 1).to(torch.uint8)
    kb = torch.cat([torch.full((n, 1), ord("t"), dtype=torch.uint8, device=dev), digits], 1).reshape(-1)
    ko = torch.arange(n + 1, device=dev, dtype=torch.int64) * 11
    # the engine runs on its own stream when torch's is the legacy default
    # one: the keys must be in HBM before it reads them
    torch.cuda.synchronize(dev)
    slots = eng.intern_device(TREG, kb, ko)
    del kb, ko, digits
    assert bool((slots == idx.to(torch.int32)).all())
    g = torch.Generator(device=dev)
    g.manual_seed(12345)

    def batch(j):
        ts = torch.randint(0, 1 << 20, (n,), device=dev, generator=g, dtype=torch.int64) + (j << 18)
        pre = torch.randint(-(1 << 62), 1 << 62, (n,), device=dev, generator=g, dtype=torch.int64)
        lr = torch.randint(1, 9, (n,), device=dev, generator=g, dtype=torch.int64)
        pad = torch.bitwise_left_shift(torch.ones_like(lr), 8 * (8 - lr)) - 1
        pre = pre & ~pad  # zero padding past the value's length
        return ts, pre, lr

    out = {}
    for form in ("block", "keyed"):
        times = []
        for j in range(steps + 2):
            ts, pre, lr = batch(j + (0 if form == "block" else 100))
            torch.cuda.synchronize(dev)
            eng.timing(True)
            if form == "block":
                eng.treg_converge_block(0, ts, pre, lr)
            else:
                eng.treg_converge(slots, ts, pre, lr)
            eng.sync()
            t = eng.timing_read()
            eng.timing(False)
            if j >= 2:
                times.append(float(np.sum(t)))
        ms = float(np.mean(times))
        out[form] = ms
        print(f"{form}: {ms:.4f} ms per call  frac(48 B/key) {48 * n / (ms * 1e-3) / 8e12:.3f}  "
              f"runs {' '.join(f'{x:.3f}' for x in times)}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
