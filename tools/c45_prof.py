"""Configs 4 and 5 alone (bench.py's legs, same arguments), for host-phase profiles:
TSG_PROF=1 python tools/c45_prof.py [bench.py options] prints the libtsg phase table at exit
covering only these two legs' calls. One JSON line: {"cfg4": ..., "cfg5": ...}."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    args = bench.parse()
    import torch
    torch.cuda.set_device(0)  # (torch's HIP runtime first, as in bench.py)
    import tempo_amd as T
    eng = T.Engine(devices=[0])
    wd = args.workdir or tempfile.mkdtemp(prefix="c45_")
    out = {}
    node = eng.numa_node(0)
    if args.pin == "auto" and node >= 0:
        os.sched_setaffinity(0, set(bench.idlest(sorted(bench.node_cpus(node) & os.sched_getaffinity(0)), 16)))
    if args.cfg4 is None or args.cfg4:
        out["cfg4"], _ = bench.cfg4_leg(args, eng, wd, 0)
    if args.cfg5:
        out["cfg5"], _ = bench.cfg5_leg(args, eng, wd, 0, 1, None)
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
