"""Build libmlic_hip.so in-tree for gfx950 (hipcc via the csrc Makefile)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs: int = 8, verbose: bool = False) -> str:
    csrc = os.path.join(HERE, "csrc")
    cmd = ["make", "-C", csrc, f"-j{jobs}", "OUT=" + os.path.join(HERE, "libmlic_hip.so")]
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError("building libmlic_hip.so failed")
    return os.path.join(HERE, "libmlic_hip.so")


if __name__ == "__main__":
    print(build(verbose=True))
