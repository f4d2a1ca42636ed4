#!/usr/bin/env python3
"""Summaries of rocprofv3's rocpd database output (ROCm 7.2 writes `<name>_results.db`, SQLite;
no CSV unless asked): per-kernel dispatch statistics as `--stats` prints them, the dispatches of
one kernel in order, and the PMC counter value of each of those dispatches.

    tools/rpd_summary.py stats DB                   # calls / total / avg / min / max per kernel
    tools/rpd_summary.py list DB SUBSTR             # every dispatch of kernels matching SUBSTR
    tools/rpd_summary.py pmc DB SUBSTR              # + the counter values per dispatch
"""
import sqlite3
import sys


def rows(db, substr=None):
    c = sqlite3.connect(db)
    q = ("select d.id, s.kernel_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x, d.event_id "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    out = [r for r in c.execute(q) if substr is None or substr in r[1]]
    return c, out


def stats(db):
    _, rs = rows(db)
    agg = {}
    for _, name, st, en, *_ in rs:
        a = agg.setdefault(name, [])
        a.append((en - st) / 1e3)
    print("%-90s %7s %12s %10s %10s %10s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us"))
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%-90s %7d %12.1f %10.2f %10.2f %10.2f" % (name[:90], len(d), sum(d), sum(d) / len(d), min(d), max(d)))


def listing(db, substr, with_pmc=False):
    c, rs = rows(db, substr)
    pmc = {}
    if with_pmc:
        names = {i: n for i, n in c.execute("select id, name from rocpd_info_pmc")}
        for ev, pid, val in c.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
            d = pmc.setdefault(ev, {})
            d[names.get(pid, pid)] = d.get(names.get(pid, pid), 0) + val
    t0 = rs[0][2] if rs else 0
    for i, (_, name, st, en, grid, wg, ev) in enumerate(rs):
        extra = " ".join("%s=%.0f" % kv for kv in sorted(pmc.get(ev, {}).items()))
        print("%4d start+%10.1f us dur %10.2f us grid %7d wg %4d %s" % (i, (st - t0) / 1e3, (en - st) / 1e3, grid, wg, extra))


if __name__ == "__main__":
    cmd, db = sys.argv[1], sys.argv[2]
    if cmd == "stats":
        stats(db)
    else:
        listing(db, sys.argv[3], with_pmc=cmd == "pmc")
