"""Build libketogpu.so (HIP for gfx950 + host C++) in-tree with hipcc.

    python -m keto_amd.build            # builds keto_amd/libketogpu.so
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libketogpu.so")
SYNTH_LIB = os.path.join(HERE, "libketosynth.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KETOGPU_ARCH", "gfx950")

SOURCES = ["snapshot.cpp", "snapshot_write.cpp", "snapshot_io.cpp", "host_engine.cpp", "multi_engine.cpp", "shard.cpp", "device_engine.hip", "partition.hip", "comm.cpp", "part_round.cpp", "tier.cpp", "core_index.cpp", "labels.cpp", "probe.hip"]
HEADERS = ["ketogpu_internal.hpp", "device_util.hpp", "part_round.hpp", "tier.hpp", "core_index.hpp", "labels.hpp", os.path.join("..", "..", "include", "ketogpu.h")]


def kernel_source_hash():
    """hash of the traversal kernels' sources.  A PMC traffic summary records the hash it
    was profiled at (tools/pmc_traffic.py); bench.py reports its traffic only while the
    hash still matches, so a stale figure never passes as current."""
    import hashlib
    h = hashlib.sha256()
    for f in ("device_engine.hip", "device_util.hpp", "core_index.hpp", "core_index.cpp", "labels.hpp", "labels.cpp"):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _stale(out, deps):
    deps = list(deps) + [os.path.abspath(__file__)]  # flag changes rebuild
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(force=False, jobs=4):
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    objs = []
    procs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            # the kernels aggregate their atomics per wave by hand (ballot + one leader);
            # the compiler's atomic optimizer only adds scalar loops (5% on the bidi kernel)
            cmd = [HIPCC, "-c", "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
                   "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
                   "-I", os.path.join(ROOT, "include"), s, "-o", o]
            if src.endswith(".cpp"):
                cmd = [HIPCC, "-c", "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
                       "-I", os.path.join(ROOT, "include"), s, "-o", o]
            print("+", " ".join(cmd), flush=True)
            procs.append(subprocess.Popen(cmd))
            if len(procs) >= jobs:
                for p in procs:
                    if p.wait():
                        raise SystemExit(f"compile failed: {p.args}")
                procs = []
    for p in procs:
        if p.wait():
            raise SystemExit(f"compile failed: {p.args}")
    if force or _stale(LIB, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs +
             ["-Wl,-rpath,/opt/rocm/lib", "-lpthread"])
    synth_src = os.path.join(CSRC, "synth.cpp")
    if os.path.exists(synth_src) and (force or _stale(SYNTH_LIB, [synth_src])):
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-o", SYNTH_LIB, synth_src, "-lpthread"])
    return LIB


def build_variant(name, defines, jobs=4):
    """libketogpu built with extra -D flags on the device sources, for A/B measurements
    (keto_amd/variants/libketogpu_<name>.so; select it with KETOGPU_LIB)"""
    build(jobs=jobs)
    objdir = os.path.join(HERE, "build", "v_" + name)
    os.makedirs(objdir, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    objs = []
    for src in SOURCES:
        if src.endswith(".cpp"):
            objs.append(os.path.join(HERE, "build", src + ".o"))
            continue
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src + ".o")
        objs.append(o)
        if _stale(o, [s] + hdrs):
            _run([HIPCC, "-c", "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-mllvm",
                  "-amdgpu-atomic-optimizer-strategy=None", "-I", os.path.join(ROOT, "include")] + list(defines) +
                 [s, "-o", o])
    out = os.path.join(HERE, "variants", f"libketogpu_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if _stale(out, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs +
             ["-Wl,-rpath,/opt/rocm/lib", "-lpthread"])
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
