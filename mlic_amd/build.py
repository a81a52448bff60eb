"""Build libmlic_hip.so in-tree for gfx950 (hipcc via the csrc Makefile) and record what was built.

The library is git-ignored but travels with the tree to the GPU box prebuilt, so every build writes
`libmlic_hip.build.json` beside it: a digest of every source it is built from (csrc/*, csrc/ab/*,
include/mlic_hip.h, the Makefile), the library's own sha256, the hipcc version and the target.
`_lib.lib()` recomputes the source digest when it loads the library and refuses a library whose
record does not match the sources in the tree (a stale or foreign build fails loudly instead of
running)."""
import datetime
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libmlic_hip.so")
RECORD = os.path.join(HERE, "libmlic_hip.build.json")


def source_files():
    csrc = os.path.join(HERE, "csrc")
    out = []
    for d in (csrc, os.path.join(csrc, "ab")):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile":
                out.append(os.path.join(d, f))
    out.append(os.path.join(ROOT, "include", "mlic_hip.h"))
    return out


def source_digest() -> str:
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, ROOT).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def build(jobs: int = 8, verbose: bool = False, incremental: bool = None) -> str:
    """Compile the library.  By default from clean (the object directory is removed first, ~90 s on 8
    cores), so the record proves that the sources of this tree compile into this library; the
    developer loop passes incremental=True (or sets $MLIC_BUILD_INCREMENTAL=1) and make rebuilds only
    what changed.  The record says which it was and how many objects were compiled."""
    import shutil
    import time
    if incremental is None:
        incremental = os.environ.get("MLIC_BUILD_INCREMENTAL", "0") not in ("", "0")
    csrc = os.path.join(HERE, "csrc")
    objdir = os.path.join(csrc, "build")
    if not incremental and os.path.isdir(objdir):
        shutil.rmtree(objdir)
    cmd = ["make", "-C", csrc, f"-j{jobs}", "OUT=" + LIB]
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if verbose:
        sys.stdout.write(r.stdout or "")
        sys.stderr.write(r.stderr or "")
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError("building libmlic_hip.so failed")
    compiled = sum(1 for ln in (r.stdout or "").splitlines() if " -c " in ln and "hipcc" in ln)
    linked = any("-shared" in ln for ln in (r.stdout or "").splitlines())
    try:
        hipcc = subprocess.run(["/opt/rocm/bin/hipcc", "--version"], capture_output=True, text=True).stdout
        hipcc = next((ln.strip() for ln in hipcc.splitlines() if "HIP version" in ln), hipcc.strip()[:80])
    except OSError:
        hipcc = "unknown"
    rec = {"library": os.path.basename(LIB), "library_sha256": _sha256(LIB), "sources_sha256": source_digest(),
           "sources": [os.path.relpath(p, ROOT) for p in source_files()], "target": "gfx950",
           "make": " ".join(cmd[:1] + cmd[3:]), "hipcc": hipcc,
           "from_clean": not incremental, "objects_compiled": compiled, "objects_total": _objects_total(csrc),
           "linked": linked, "build_seconds": round(time.time() - t0, 1),
           "built_at": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds")}
    with open(RECORD, "w") as f:
        json.dump(rec, f, indent=1)
    return LIB


def _objects_total(csrc: str) -> int:
    r = subprocess.run(["make", "-C", csrc, "-p", "-n", "-q"], capture_output=True, text=True)
    for ln in (r.stdout or "").splitlines():
        if ln.startswith("SRCS = ") or ln.startswith("SRCS := "):
            return len(ln.split("=", 1)[1].split())
    return -1


if __name__ == "__main__":
    print(build(verbose=True, incremental="--incremental" in sys.argv))
