"""Which sources a measurement belongs to: a hash of the product's kernel and host sources.

The GPU box receives the source tree without git history, so profiles (tools/profile.sh)
and bench.py identify the code they ran by this hash instead of a commit id: bench.py only
replays a profile's counters (roofline.traffic, executed VALU) when the hashes agree."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files():
    pats = ["rust_tracer_amd/csrc/*.hip", "rust_tracer_amd/csrc/*.hpp", "rust_tracer_amd/csrc/*.cpp",
            "rust_tracer_amd/csrc/Makefile", "include/*.h"]
    files = []
    for p in pats:
        files += glob.glob(os.path.join(ROOT, p))
    return sorted(files)


def sources_sha():
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()[:16]
