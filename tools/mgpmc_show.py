"""Print the SQ / traffic counters of tools/gpu_mgpmc.sh per kernel."""
import json
import sys

d = sys.argv[1]
out = {}
for p in "ABFW":
    try:
        s = json.load(open(f"{d}/pmc{p}_summary.json"))
    except FileNotFoundError:
        continue
    for k, v in s.items():
        out.setdefault(k, {}).update({n: x["mean"] for n, x in v.items()})
for k, v in out.items():
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    g = lambda n: v.get(n, 0)
    w = g("SQ_WAVES") or 1
    print(k)
    print("  waves %d VALU/w %.0f LDS/w %.0f SALU/w %.0f VMEMRD/w %.1f VMEMWR/w %.1f" % (
        w, g("SQ_INSTS_VALU") / w, g("SQ_INSTS_LDS") / w, g("SQ_INSTS_SALU") / w, g("SQ_INSTS_VMEM_RD") / w,
        g("SQ_INSTS_VMEM_WR") / w))
    print("  wavecyc %.0f waitany %.0f activeany %.0f valu %.0f lds %.0f waitlds %.0f bankconf %.0f" % tuple(
        g(n) for n in ["SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                       "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT"]))
    print("  fetch MB %.1f write MB %.1f" % (g("FETCH_SIZE") / 1024, g("WRITE_SIZE") / 1024))
