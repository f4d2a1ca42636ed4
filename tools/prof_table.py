"""Summarise TSG_PROF output: per labelled table (tsgx_prof_flush), the p50 of the named phases.
python tools/prof_table.py <stderr file> <phase> ..."""
import re
import sys


def main():
    path, names = sys.argv[1], sys.argv[2:]
    label = None
    for line in open(path, errors="replace"):
        m = re.match(r"\[tsg\] prof \[(.*)\]", line)
        if m:
            label = m.group(1)
            continue
        if line.startswith("[tsg] prof p50 us:"):
            vals = dict(re.findall(r" ([\w.]+)=([0-9.]+)", line))
            print("%-20s" % (label or "(exit)"), " ".join("%s=%s" % (n, vals[n]) for n in names if n in vals))
            label = None


if __name__ == "__main__":
    main()
