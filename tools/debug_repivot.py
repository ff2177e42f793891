import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "sharedmemsparselu.jl_amd"))
import numpy as np, scipy.sparse as sp
import smlu

def run(tag, D, env):
    for k, v in env.items():
        os.environ[k] = v
    try:
        F = smlu.ParallelSparseLU(sp.csc_matrix(D))
        b = np.random.default_rng(1).random(D.shape[0]); x = np.empty_like(b)
        smlu.ldiv_(x, F, b)
        err = np.linalg.norm(D @ x - b) / np.linalg.norm(b)
        print(tag, "ok resid", err, "repivots", F.stat("repivots"), "pivmode", F.stat("pivmode"),
              "tall", F.stat("launches_panel_tall"), "mode1", F.stat("fronts_mode1"), "mode2", F.stat("fronts_mode2"), flush=True)
    except Exception as e:
        print(tag, "EXC", e, flush=True)
    for k in env:
        del os.environ[k]

rng = np.random.default_rng(17)
D = rng.random((700, 700))
run("rand700 mode1-forced", D, {"SMLU_FULLPIV_NS": "100000"})
run("rand520 mode1-forced", rng.random((520, 520)), {"SMLU_FULLPIV_NS": "100000"})
run("rand600 mode1-forced", rng.random((600, 600)), {"SMLU_FULLPIV_NS": "100000"})
Z = D.copy(); Z[:64, :64] = 0
run("zero-tile mode1-forced", Z, {"SMLU_FULLPIV_NS": "100000"})
run("zero-tile default", Z, {})
Z2 = D.copy(); Z2[100:164, 100:164] = 0
run("zero-tile@100 default", Z2, {})
