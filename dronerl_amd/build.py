"""Build libdronerl.so (hand-written HIP for gfx950) in-tree with hipcc.

python -m dronerl_amd.build   (or dronerl_amd.build.build())
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdronerl.so")
HASH = LIB + ".srchash"
SOURCES = [os.path.join(CSRC, "dronerl_kernels.hip"), os.path.join(CSRC, "dronerl_api.cpp"),
           os.path.join(CSRC, "dronerl_env.cpp"), os.path.join(CSRC, "dronerl_qnet.hip"),
           os.path.join(CSRC, "dronerl_qnet_api.cpp"), os.path.join(CSRC, "dronerl_learn.hip")]
DEPS = SOURCES + [os.path.join(CSRC, "dronerl_internal.h"), os.path.join(REPO, "include", "dronerl.h")]
ARCH = os.environ.get("DRL_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in [os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"]:
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]


def compile_cmd(out: str):
    """The whole library in one hipcc command (tools/variants.py's form)."""
    return [hipcc(), f"--offload-arch={ARCH}"] + FLAGS + ["-shared", "-I", os.path.join(REPO, "include"),
                                                         "-o", out] + SOURCES


def object_cmd(src: str, obj: str):
    """One translation unit (host + gfx950 device code) -> an object; every kernel is launched from its own
    unit, so the units link as they are (no relocatable device code)."""
    return [hipcc(), f"--offload-arch={ARCH}"] + FLAGS + ["-c", "-I", os.path.join(REPO, "include"), "-o", obj, src]


def source_digest() -> str:
    """sha256 over every source/header the library is built from and the
    target arch: the key a built library is checked against."""
    h = hashlib.sha256(ARCH.encode())
    for d in DEPS:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def up_to_date() -> bool:
    try:
        with open(HASH) as f:
            return os.path.exists(LIB) and f.read().strip() == source_digest()
    except OSError:
        return False


def build(force: bool = False, verbose: bool = False) -> str:
    """Rebuild unless the library on disk was built from exactly these sources
    (its sidecar LIB.srchash holds their digest; _native refuses to load a
    library whose digest does not match the sources beside it)."""
    if not force and up_to_date():
        return LIB
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    digest = source_digest()
    with tempfile.TemporaryDirectory(prefix="drl_build_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(src) + ".o") for src in SOURCES]
        cmds = [object_cmd(src, obj) for src, obj in zip(SOURCES, objs)]
        if verbose:
            for c in cmds:
                print(" ".join(c), file=sys.stderr)
        # the units compile in parallel (the kernels' unit dominates the wall time)
        with ThreadPoolExecutor(max(1, min(len(cmds), os.cpu_count() or 1))) as ex:
            for r in ex.map(lambda c: subprocess.run(c, capture_output=not verbose, text=True), cmds):
                if r.returncode:
                    if not verbose:  # (the compiler's messages, which were captured)
                        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
                    raise subprocess.CalledProcessError(r.returncode, r.args, r.stdout, r.stderr)
        link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp"] + objs
        if verbose:
            print(" ".join(link), file=sys.stderr)
        subprocess.run(link, check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(HASH, "w") as f:
        f.write(digest + "\n")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
