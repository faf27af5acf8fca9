"""Reader of the canonical descriptor dumps (skirt_host_write_descriptors, include/skirt_host.h)."""
import numpy as np

_TYPES = {"d": np.float64, "i": np.int32, "b": np.int8}


def read(path):
    """{field name: numpy array} of a dump; a field written twice is an error"""
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        end = data.index(b"\n", pos)
        name, typ, count = data[pos:end].decode().split()
        dt = np.dtype(_TYPES[typ])
        n = int(count)
        pos = end + 1
        arr = np.frombuffer(data, dtype=dt, count=n, offset=pos).copy()
        pos += n * dt.itemsize
        assert name not in out, name
        out[name] = arr
    return out


def differences(a, b):
    """the fields of two dumps that are not bit for bit equal (missing on one side included)"""
    diffs = []
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            diffs.append((k, "only in " + ("first" if k in a else "second")))
        elif a[k].shape != b[k].shape:
            diffs.append((k, "lengths %d and %d" % (a[k].size, b[k].size)))
        elif a[k].tobytes() != b[k].tobytes():
            bytes_a = a[k].view(np.uint8).reshape(a[k].size, -1)
            bytes_b = b[k].view(np.uint8).reshape(b[k].size, -1)
            bad = np.flatnonzero(np.any(bytes_a != bytes_b, axis=1))
            diffs.append((k, "%d of %d values differ, first at %d: %r vs %r" %
                          (bad.size, a[k].size, bad[0], a[k][bad[0]], b[k][bad[0]])))
    return diffs
