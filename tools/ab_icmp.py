#!/usr/bin/env python3
"""Same-process A/B of the ICMP echo-reflect launch (bench.py icmp line) over
library builds: usage: ab_ev.py LIB1,LIB2,... [ROUNDS]. Each build's result
is also checked against the oracle (bench.parity_leg)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ix_amd import ixgrx, traces
    libs = sys.argv[1].replace("+", ",").split(",")
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    res = {}
    for _ in range(rounds):
        for lib in libs:
            engs = {}

            def eng_for(flags, lib=lib, engs=engs):
                if flags not in engs:
                    engs[flags] = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, flags), device=0,
                                                 lib_path=os.path.join(ROOT, lib))
                return engs[flags]
            line, chk = bench.icmp_line(dev, 10, 0, eng_for)
            par = bench.parity_leg([chk], traces.RSS_KEY)["icmp"]
            r = res.setdefault(os.path.basename(lib), {"ms": [], "parity": []})
            r["ms"].append(line["kernel_ms_avg"])
            r["parity"].append(par)
            for e in engs.values():
                e.close()
            torch.cuda.empty_cache()
    print(json.dumps({k: {"min_ms": min(v["ms"]), "ms": v["ms"], "parity": sorted(set(v["parity"]))}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
