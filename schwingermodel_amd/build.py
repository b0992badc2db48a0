"""In-tree build of libsm_hip.so for gfx950 (hipcc; no JIT cache, no pip install).

    python schwingermodel_amd/build.py          # library + sm_hmc (not -m: the package import loads the old .so)
The .so lands next to this file, so it travels with the repo snapshot to the
GPU box and is the one the tests / bench / smoke load.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libsm_hip.so")
SOURCES = ["sm_kernels.hip", "sm_cgfused.hip", "sm_cgra.hip", "sm_eotd.hip", "sm_gauge.hip", "sm_eo.hip", "sm_peer.hip", "sm_capi.cpp", "sm_comm.cpp", "sm_place.cpp", "sm_conf.cpp", "sm_md.cpp", "sm_hmc.cpp",
           "sm_eo.cpp"]
HEADERS = ["sm_internal.h", "sm_fields.h", "sm_device.h", "sm_ctx.h", "sm_linkcode.h", "sm_peer.h"]

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("SM_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: no FMA contraction, so D / D^dag / force are bit-identical
# to the reference's x86-64 (non-FMA) std::complex arithmetic.
CFLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Wall",
          f"--offload-arch={ARCH}", f"-I{ROCM}/include", f"-I{os.path.join(REPO, 'include')}"]
LDFLAGS = ["-shared", f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def source_id():
    """Build id of the library: SHA-256 (16 hex) of its sources, headers and
    compile flags. Compiled into the library (sm_build_id()) so a profile
    summary recorded with one build can be matched to the build that runs
    (bench.py's roofline.traffic_source), independent of whether the compiler
    output is byte-reproducible."""
    import hashlib
    h = hashlib.sha256()
    for name in SOURCES + HEADERS:
        h.update(name.encode())
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    with open(os.path.join(REPO, "include", "sm_hip.h"), "rb") as f:
        h.update(f.read())
    h.update(" ".join(CFLAGS + LDFLAGS).encode())
    return h.hexdigest()[:16]


def build_library(force=False, verbose=True):
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(REPO, "include", "sm_hip.h"))
    if not force and not _stale(LIB, deps):
        return LIB
    if not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    # one hipcc per translation unit, in parallel (objects under build/, git-ignored),
    # then one link; a source whose object is newer than it and every header is reused
    objdir = os.path.join(REPO, "build", "sm_hip")
    os.makedirs(objdir, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "sm_hip.h")]
    jobs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(objdir, s + ".o")
        if force or _stale(obj, [src] + hdrs):
            jobs.append([HIPCC] + CFLAGS + ["-c", src, "-o", obj])
    from concurrent.futures import ThreadPoolExecutor
    nproc = min(len(jobs) or 1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with ThreadPoolExecutor(nproc) as ex:
        procs = list(ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs))
    for c, p in zip(jobs, procs):
        if verbose or p.returncode:
            print(" ".join(c), file=sys.stderr)
            sys.stderr.write(p.stderr)
        if p.returncode:
            raise subprocess.CalledProcessError(p.returncode, c)
    bid_src = os.path.join(objdir, "sm_build_id.cpp")
    with open(bid_src, "w") as f:
        f.write(f'extern "C" const char *sm_build_id(void) {{ return "{source_id()}"; }}\n')
    bid_obj = bid_src + ".o"
    subprocess.run(["g++", "-O2", "-fPIC", "-c", bid_src, "-o", bid_obj], check=True)
    tmp = LIB + ".tmp"
    cmd = ([HIPCC, f"--offload-arch={ARCH}"] + [os.path.join(objdir, s + ".o") for s in SOURCES] + [bid_obj]
           + ["-o", tmp] + LDFLAGS)
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


CLI = os.path.join(HERE, "sm_hmc")
MPI_ROOT = os.environ.get("SM_MPI_ROOT", "/opt/conda")


def build_cli(force=False, verbose=True):
    """`sm_hmc`: the reference's HMC program (src/main.cpp) on the device
    layer, one MPI rank per GPU. Needs an MPI (the image's MPICH under
    /opt/conda, as the reference); skipped with a note when absent."""
    src = os.path.join(CSRC, "sm_hmc_main.cpp")
    mpi_so = os.path.join(MPI_ROOT, "lib", "libmpi.so")
    if not os.path.exists(os.path.join(MPI_ROOT, "include", "mpi.h")) or not os.path.exists(mpi_so):
        print(f"sm_hmc not built: no MPI under {MPI_ROOT}", file=sys.stderr)
        return None
    if not force and not _stale(CLI, [src, LIB, os.path.join(REPO, "include", "sm_hip.h")]):
        return CLI
    cmd = ["g++", "-O2", "-std=c++17", f"-I{os.path.join(REPO, 'include')}", f"-I{MPI_ROOT}/include", src,
           "-o", CLI + ".tmp", mpi_so, f"-Wl,-rpath,{MPI_ROOT}/lib", "-static-libstdc++", "-static-libgcc",
           # conda's old libstdc++ must not shadow the system one libsm_hip.so needs
           "-Wl,-rpath-link,/usr/lib/x86_64-linux-gnu", f"-Wl,-rpath-link,{ROCM}/lib",
           f"-L{HERE}", "-lsm_hip", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(CLI + ".tmp", CLI)
    return CLI


def build_oracle(with_reference=None):
    """Test checker: oracle/liboracle.so, plus oracle/_ref/ when /root/reference exists."""
    oracle_dir = os.path.join(REPO, "oracle")
    subprocess.run(["make", "-s", "-C", oracle_dir, "oracle"], check=True)
    if with_reference is None:
        with_reference = os.path.isdir("/root/reference/src")
    if with_reference and shutil.which("g++"):
        subprocess.run(["make", "-s", "-C", oracle_dir, "ref"], check=True)
        # the reference's own driver code linked against our drop-in shim
        subprocess.run(["make", "-s", "-C", oracle_dir, "dropin", "refapp"], check=True)


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
    build_cli(force="--force" in sys.argv)
