"""Classify ThreadSanitizer reports by where each racing access happens.

For both accesses of a report the first frame outside TSan's own interceptors (operator
new/delete, memcpy, free, ...) is taken as the access site.  A report counts against this
repository only when one of those sites is a frame in its sources (blb_amd/, tests/cpp/);
a race whose accesses are both inside an uninstrumented library (the ROCm runtime) is
reported by library.

usage: python tools/tsan_summary.py rs_test_tsan.log[.gz]
"""
from __future__ import annotations

import collections
import gzip
import re
import sys

_ACCESS = re.compile(r"^  (Previous )?(atomic )?(read|write) of size", re.I)
_FRAME = re.compile(r"^    #(\d+) (.*) \(([^ ()]+)\+0x[0-9a-f]+\)")


def _site(frames):
    for text, mod in frames:
        if "compiler-rt/lib/tsan" in text or "sanitizer_common" in text:
            continue
        if "/root/repo/" in text:
            return "repo:" + text.split("/root/repo/")[1].split()[0]
        return mod.rsplit("/", 1)[-1]
    return "?"


def _caller(frames):
    """The innermost frame in this repository's sources (the call that entered the runtime)."""
    for text, _ in frames:
        if "/root/repo/" in text:
            return text.split("/root/repo/")[1].split()[0]
    return "(runtime thread)"


def main(path: str) -> None:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rt", errors="replace") as f:
        lines = f.read().splitlines()
    reports, cur, stack = [], None, None
    for ln in lines:
        if ln.startswith("WARNING: ThreadSanitizer"):
            cur = {"kind": ln.split(": ", 1)[1].split(" (")[0], "sites": []}
            reports.append(cur)
            stack = None
        elif cur is not None and _ACCESS.match(ln):
            stack = []
            cur["sites"].append(stack)
        elif cur is not None and ln.startswith("  ") and not ln.startswith("    "):
            stack = None                       # mutex / thread creation sections
        elif stack is not None:
            m = _FRAME.match(ln)
            if m:
                stack.append((m.group(2), m.group(3)))
    by_pair, by_caller = collections.Counter(), collections.Counter()
    ours = []
    for r in reports:
        sites = tuple(sorted(_site(s) for s in r["sites"]))
        by_pair[(r["kind"],) + sites] += 1
        by_caller[tuple(sorted(_caller(s) for s in r["sites"]))] += 1
        if any(s.startswith("repo:") for s in sites):
            ours.append(sites)
    print(f"{len(reports)} reports; racing accesses (innermost frame outside TSan):")
    for key, n in by_pair.most_common():
        print(f"{n:5d}  {key[0]}: " + "  <->  ".join(key[1:]))
    print("the calls into the runtime they happened under (innermost frame in this repository):")
    for key, n in by_caller.most_common():
        print(f"{n:5d}  " + "  <->  ".join(key))
    print(f"reports with an access in this repository's code: {len(ours)}")
    for s in ours[:20]:
        print("   ", s)


if __name__ == "__main__":
    main(sys.argv[1])
