import sys, json, time
sys.path.insert(0, '.')
import quant_amd
eng = quant_amd.Engine(0)
for (S, bw, bits) in [(512, 2, 10), (4096, 2, 10), (4096, 4, 12)]:
    eng.set_synthetic(S, 0x5EED, 1, bw, bw)
    for rep in range(3):
        t = time.time(); C, A, d = eng.lbg(bits, want_assign=False); dt = time.time() - t
    tm = eng.timings()
    print(json.dumps({"S": S, "bw": bw, "bits": bits, "wall_s": dt, "total_ms": tm["total_ms"],
                      "assign_ms": [round(x, 4) for x in tm["assign_ms"]], "update_ms": [round(x, 4) for x in tm["update_ms"]],
                      "flagged": tm["flagged"], "host_ties": tm["host_ties"]}), flush=True)
