"""A benchmark model (benchmarks/*.ski) as the bench fixtures run it: 1e3 packages per wavelength and the
diagnostic outputs on (ds_convergence, ds_crossed, ds_cellprops). Test infrastructure.
usage: python bench_ski.py <benchmarks/cN.ski>   (writes the variant to stdout)"""
import re
import sys

PACKAGES = "1e3"


def variant(text):
    text = re.sub(r'packages="[^"]*"', 'packages="%s"' % PACKAGES, text, count=1)
    for prop in ("writeConvergence", "writeCellsCrossed", "writeCellProperties"):
        text = re.sub(r'%s="[^"]*"' % prop, '%s="true"' % prop, text)
    return text


if __name__ == "__main__":
    sys.stdout.write(variant(open(sys.argv[1]).read()))
