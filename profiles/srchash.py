"""The source hash a PMC profile is keyed by: sha256 over the engine's
kernel sources — every csrc/*.hip and csrc/*.hpp of the package and the C ABI headers
(include/*.h) —
so a profile describes exactly the code that ran.  profiles/summarize_legs.py stamps each
entry of pmc_legs.json with it (computed on the GPU box from the tree that was profiled);
bench.py attaches a leg's traffic only when the stamp equals the hash of the tree it runs
from, so any change to a kernel retires every profile taken before it."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "compressed-fm-index-implementation-with-learned-optimizations_amd")


def kernel_src_hash() -> str:
    files = sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")) + glob.glob(os.path.join(PKG, "csrc", "*.hpp")))
    files += sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(kernel_src_hash())
