"""Debug aid: replay a random TLOG history through the engine and the oracle,
stop at the first converge whose result differs, and dump that step."""
import sys, os, pickle
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import numpy as np
import oracle
from helpers import random_history
from jylis_amd.engine import Engine
from jylis_amd.repo import RepoTLOG

oracle.load()
O = oracle
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
want = O.Repo(O.TLOG)
eng = Engine(device=0)
got = RepoTLOG(eng)
prev = None
for n, b in enumerate(random_history(O, O.TLOG, seed, nops=400, val_len=20)):
    before = want.state()
    want.converge(b)
    got.converge_deltas(b)
    w, g = want.state(), got.state()
    same = set(w) == set(g) and all(np.array_equal(np.asarray(w[k]), np.asarray(g[k])) for k in w)
    if not same:
        nent = len(b["ts"])
        print("diverged at batch", n, "keys", len(b["cutoff"]), "entries", nent)
        with open("gpurun_out/tlog_div.pkl", "wb") as f:
            pickle.dump({"n": n, "batch": b, "before": before, "want": w, "got": g}, f)
        break
else:
    print("no divergence")
eng.close()
