"""Build the native pieces in-tree (no JIT caches, so the .so files travel to the GPU box).

- openmavis_amd/libomv_hip.so : the product — hand-written gfx950 HIP kernels + the C ABI of
  include/omv.h (hipcc --offload-arch=gfx950, -ffp-contract=off for the bit-exact float paths).
- oracle/liboracle.so          : test infrastructure — the CPU restatement used as checker and as
  bench.py's cpu_baseline leg (built with g++, never linked into the product).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "openmavis_amd")
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libomv_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OMV_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["orb_extract.hip", "match.hip", "lba.hip", "pose.hip", "tri.hip", "frame.hip", "imu.hip", "bow.hip", "bowmatch.hip",
               "mappoint.hip", "fuse.hip"]
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
             f"--offload-arch={ARCH}", "-Wno-unused-result"]
OBJ_DIR = os.path.join(ROOT, "build", "obj")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_hip(force=False, verbose=True, defines=(), lib=LIB, obj_dir=OBJ_DIR):
    """One hipcc -c per translation unit (in parallel, only the stale ones), then one shared link.
    `defines` / `lib` / `obj_dir` build an instrumented variant (e.g. -DOMV_RESOLVE_PROFILE) beside the product."""
    from concurrent.futures import ThreadPoolExecutor
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES if os.path.exists(os.path.join(CSRC, s))]
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".inc"))]
    hdrs.append(os.path.join(ROOT, "include", "omv.h"))
    os.makedirs(obj_dir, exist_ok=True)
    objs = [os.path.join(obj_dir, os.path.basename(s) + ".o") for s in srcs]
    stale = [(s, o) for s, o in zip(srcs, objs) if force or _newer(o, [s] + hdrs)]

    def compile_one(so):
        s, o = so
        cmd = [HIPCC] + HIP_FLAGS + [f"-D{d}" for d in defines] + ["-I", os.path.join(ROOT, "include"), "-c", s, "-o", o + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(o + ".tmp", o)

    if stale:
        with ThreadPoolExecutor(max_workers=min(8, len(stale))) as ex:
            list(ex.map(compile_one, stale))
    if not stale and not _newer(lib, objs):
        return lib
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", lib + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


def build_variant(name, defines, verbose=True):
    """Instrumented library openmavis_amd/variants/libomv_<name>.so (timing printfs etc.; never the product)."""
    vdir = os.path.join(PKG, "variants")
    os.makedirs(vdir, exist_ok=True)
    return build_hip(False, verbose, defines, os.path.join(vdir, f"libomv_{name}.so"),
                     os.path.join(ROOT, "build", "obj_" + name))


def build_oracle(verbose=True):
    odir = os.path.join(ROOT, "oracle")
    subprocess.check_call(["make", "-s", "-C", odir], stdout=None if verbose else subprocess.DEVNULL)
    return os.path.join(odir, "liboracle.so")


CONSUMER_SRC = os.path.join(ROOT, "tests", "cpp", "omv_consumer.cpp")
CONSUMER_BIN = os.path.join(PKG, "bin", "omv_consumer")


def build_consumer(verbose=True):
    """tests/cpp/omv_consumer.cpp: a plain C++ (g++) consumer of include/omv.h + include/omv_adapters.hpp, linked
    against libomv_hip.so and the HIP runtime only (test infrastructure for the C++ integration path)."""
    deps = [CONSUMER_SRC, os.path.join(ROOT, "include", "omv.h"), os.path.join(ROOT, "include", "omv_adapters.hpp"), LIB]
    if not os.path.exists(CONSUMER_SRC) or not _newer(CONSUMER_BIN, deps):
        return CONSUMER_BIN
    os.makedirs(os.path.dirname(CONSUMER_BIN), exist_ok=True)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(rocm, "include"), CONSUMER_SRC,
           "-o", CONSUMER_BIN + ".tmp", "-L", PKG, "-lomv_hip", "-Wl,-rpath,$ORIGIN/..",
           "-L", os.path.join(rocm, "lib"), "-lamdhip64", "-lrccl", "-Wl,-rpath," + os.path.join(rocm, "lib")]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(CONSUMER_BIN + ".tmp", CONSUMER_BIN)
    return CONSUMER_BIN


def build_all(force=False, verbose=True):
    build_oracle(verbose)
    lib = build_hip(force, verbose)
    build_consumer(verbose)
    return lib


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "variant":   # python -m openmavis_amd.build variant NAME DEF...
        print(build_variant(sys.argv[2], sys.argv[3:]))
    else:
        build_all(force="--force" in sys.argv)
