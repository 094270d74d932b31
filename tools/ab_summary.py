#!/usr/bin/env python3
"""Summarise tools/ab.py JSON lines (from stdin or log files): median ms per build, relative to
the first build, and whether every build matched the reference."""
import json
import sys


def lines(args):
    if not args:
        yield from sys.stdin
    for p in args:
        with open(p) as f:
            yield from f


def main():
    for line in lines(sys.argv[1:]):
        line = line.strip()
        if not line.startswith("{"):
            if line:
                print(line[:200])
            continue
        d = json.loads(line)
        if "results" not in d:
            continue
        r = d["results"]
        base = next(iter(r.values()))["median_ms"]
        parts = [f"{k.replace('libceres_hip', '')}: {v['median_ms']:.4f} ({(v['median_ms'] / base - 1) * 100:+.1f}%)"
                 for k, v in r.items()]
        mode = f"batch x{d['streams']}" if d["streams"] else "solo"
        print(f"{d['config']:<20} {mode:<9} " + "  ".join(parts) + ("" if all(v["parity"] for v in r.values()) else "  PARITY FAIL"))


if __name__ == "__main__":
    main()
