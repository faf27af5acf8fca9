"""Byte comparison of two sets of reference outputs (test infrastructure).

`skirt` stamps each FITS header with its creation time (DATE card) and each log line with the wall clock;
everything else it writes is deterministic at `-t 1`. So two runs are equal when their files are byte-equal
after blanking the FITS DATE card, the log's time stamps and the phase timings ("... in 0.6 s.").
usage: python compare_ref.py <dir A> <dir B>  (every file of A must exist in B and be equal)
"""
import os
import re
import sys


def normalized(path):
    data = open(path, "rb").read()
    if path.endswith(".fits"):
        out = bytearray(data)
        end = out.find(b"END" + b" " * 77)
        for i in range(0, max(0, end), 80):
            if out[i:i + 8] == b"DATE    ":
                out[i:i + 80] = b" " * 80
        return bytes(out)
    if path.endswith("_log_excerpt.txt"):
        lines = []
        for line in data.decode().splitlines():
            line = re.sub(r"^\d\d/\d\d/\d{4} \d\d:\d\d:\d\d\.\d{3} ", "", line)
            line = re.sub(r" in [0-9.]+ s\.$", " in T s.", line)
            lines.append(line)
        return "\n".join(lines).encode()
    return data


def differing(dir_a, dir_b, prefix=""):
    """Names of the files of dir_a (starting with prefix) that are missing from dir_b or differ (files only: the
    bench/ subdirectory holds fixtures of their own, make_bench_fixtures.sh)."""
    bad = []
    for name in sorted(os.listdir(dir_a)):
        if not name.startswith(prefix) or os.path.isdir(os.path.join(dir_a, name)):
            continue
        other = os.path.join(dir_b, name)
        if not os.path.exists(other) or normalized(os.path.join(dir_a, name)) != normalized(other):
            bad.append(name)
    return bad


if __name__ == "__main__":
    bad = differing(sys.argv[1], sys.argv[2])
    print("differ:", bad if bad else "none")
    sys.exit(1 if bad else 0)
