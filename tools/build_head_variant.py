#!/usr/bin/env python3
"""Build variants/<name>.so from the sources of a git revision (default HEAD), for an
A/B against the working tree's build: build_head_variant.py [name] [rev]."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(name="head", rev="HEAD"):
    root = os.path.join("/tmp/slvar", name)
    subprocess.run(["rm", "-rf", root], check=True)
    os.makedirs(root)
    arc = subprocess.run(["git", "-C", REPO, "archive", rev, "safelife-k2_amd/csrc", "include"],
                         check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", root], input=arc, check=True)
    csrc = os.path.join(root, "safelife-k2_amd", "csrc")
    srcs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".cpp")))
    out = os.path.join(REPO, "variants")
    os.makedirs(out, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-shared", "-munsafe-fp-atomics", "-fno-gpu-rdc", "-ffp-contract=off",
                    "-DSL_BUILD_ID=\"var-%s\"" % name] + srcs + ["-o", os.path.join(out, name + ".so")],
                   check=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
