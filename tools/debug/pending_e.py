import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
from pinc_amd import configs
from pinc_amd.sim import Sim
cfg = configs.config("warm", true_size=(32, 32, 32), ppc=8, nalloc_pc=16, levels=3)
cfg["population"].update({"layout": "tiled", "sortInterval": "1", "fused": "1"})
res = {}
for mode in ("plain", "plain2", "twice", "getonly", "unfused"):
    c = dict(cfg)
    c["population"] = dict(cfg["population"])
    if mode == "unfused":
        c["population"]["fused"] = "0"
    ini = configs.write_ini(c)
    with Sim(ini, maxwell=True, perturb=False, seed=11) as s:
        s.init()
        s.op("acc")
        if mode == "getonly":
            s.grid(2)
        if mode == "twice":
            s.particles(0)
        res[mode] = [s.particles(sp) for sp in range(2)]
def cmp(a, b):
    for sp in range(2):
        pa, va = res[a][sp]
        pb, vb = res[b][sp]
        if a == "unfused" or b == "unfused":
            oa = np.lexsort(np.vstack([va.T[::-1], pa.T[::-1]])); ob = np.lexsort(np.vstack([vb.T[::-1], pb.T[::-1]]))
            pa, va, pb, vb = pa[oa], va[oa], pb[ob], vb[ob]
        dv = np.abs(va - vb)
        print(a, b, sp, "pos", np.abs(pa - pb).max(), "vel", dv.max(), "bad", int((dv.max(1) > 1e-12).sum()), flush=True)
for a, b in [("plain", "plain2"), ("plain", "twice"), ("plain", "getonly"), ("plain", "unfused"), ("getonly", "unfused")]:
    cmp(a, b)
