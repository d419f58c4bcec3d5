"""In-tree build of the ``_C`` extension: hipcc for the gfx950 kernels, g++ for the pybind11 glue.

No hipify, no torch JIT cache: ``python -m ewdml.ops.build`` (or ``__graft_entry__.build()``) writes
``ops/_C<EXT_SUFFIX>`` next to this file, so the shared object travels with the repo snapshot to
the GPU box.  Objects are rebuilt only when a source or header is newer.
"""
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
ARCH = os.environ.get("EWDML_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = [
    "-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-ffp-contract=off",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
]


def ext_path() -> str:
    return os.path.join(HERE, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + _headers())


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def build(verbose: bool = False, force: bool = False) -> str:
    import pybind11

    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    jobs = []
    objs = []
    for f in srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(BUILD, f + ".o")
        objs.append(obj)
        if not force and not _stale(obj, src):
            continue
        if f.endswith(".hip"):
            cmd = [HIPCC, "-c", *HIP_FLAGS, "-I", CSRC, "-o", obj, src]
        else:
            cmd = ["g++", "-c", "-O2", "-fPIC", "-std=c++17", "-I", CSRC,
                   "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"],
                   "-fvisibility=hidden", "-o", obj, src]
        jobs.append(cmd)
    import time

    def timed(cmd):
        t0 = time.time()
        r = _run(cmd)
        return cmd, r, time.time() - t0

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for cmd, r, dt in ex.map(timed, jobs):
            if verbose:  # one line per compiled file: the command and its wall time
                print(f"[{dt:6.1f} s] {' '.join(cmd)}", flush=True)
                if r.stdout or r.stderr:
                    print(r.stdout, r.stderr)
    out = ext_path()
    if force or jobs or not os.path.exists(out):
        link = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", out, *objs]
        _run(link)
        if verbose:
            print(" ".join(link), flush=True)
    return out


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
