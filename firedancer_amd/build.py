"""Build the MI355X (gfx950) engine and the test-infrastructure oracle, in tree.

    python -m firedancer_amd.build          # or __graft_entry__.build()

Outputs:
    firedancer_amd/libfd_ed25519_amd.so   the product: HIP kernels + C-ABI
    firedancer_amd/libfd_ed25519_amd_diag.so  (python -m firedancer_amd.build --diag) the same plus the
                                          FD_AMD_DIAG measurement aids (k_tile_synth, the pool's and the
                                          tile kernel's clocks) -- tools only, never the product
    oracle/liboracle.so                   CPU restatement (checker only)
    oracle/_ref/libfdref.so               the reference's own sources, compiled
                                          (only when /root/reference exists)
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "firedancer_amd")
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libfd_ed25519_amd.so")
LIB_DIAG = os.path.join(PKG, "libfd_ed25519_amd_diag.so")
ARCH = os.environ.get("FD_AMD_ARCH", "gfx950")

SOURCES = ["fd_ed25519_kernels.hip", "fd_txn_kernels.hip", "fd_ed25519_sign.hip", "fd_ed25519_engine.cpp", "fd_ed25519_multi.cpp", "fd_ed25519_host.cpp",
           "fd_verify_tile.cpp", "fd_numa.cpp"]
HEADERS = ["fd_ed25519_dev.h", "fd_ed25519_kernels.h", "../../include/fd_ed25519_amd.h", "../../include/fd_txn_amd.h", "../../include/fd_tango_amd.h", "fd_ed25519_engine.h",
           "../../tools/gen_consts.py"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the engine is HIP-only (no CPU build)")


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_engine(force=False, verbose=False, out=None, defines=(), vgpr_guard=True):
    """Compile every source to an object in parallel (one hipcc per file),
    then link the shared library."""
    consts = os.path.join(CSRC, "fd_ed25519_consts.h")
    gen = os.path.join(ROOT, "tools", "gen_consts.py")
    if force or _stale(consts, [gen]):
        subprocess.check_call([sys.executable, gen, consts, "FD_AMD"])
    lib = out or LIB
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [consts]
    if not force and not defines and not _stale(lib, deps):
        return lib
    objdir = os.path.join(PKG, "_obj", os.path.basename(lib).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    base = [_hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]
    base += ["-D" + d for d in defines]
    objs = [os.path.join(objdir, s + ".o") for s in SOURCES]

    def cc(k):
        cmd = base + ["-c", os.path.join(CSRC, SOURCES[k]), "-o", objs[k]]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd, cwd=CSRC)

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), max(1, min(8, os.cpu_count() or 1)))) as ex:
        list(ex.map(cc, range(len(SOURCES))))
    n = loop_spill_stores(objs[0], TILE_KERNEL) if vgpr_guard else 0
    if n is None:   # fail closed: a build whose tile kernel cannot be inspected is not shipped
        raise RuntimeError("cannot inspect k_tile_persist for in-loop VGPR spills (the LLVM tools under "
                           "/opt/rocm/lib/llvm/bin are missing, or the kernel symbol %s is not in the code "
                           "object): refusing the build; see profiles/r05_scout_stop_cause.txt" % TILE_KERNEL)
    if n:
        raise RuntimeError("k_tile_persist spills VGPRs to scratch inside its persistent loop (%d scratch stores after "
                           "the first s_sleep): every such build lost its scout wave on hardware; see "
                           "profiles/r05_scout_stop_cause.txt" % n)
    cmd = [_hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib + ".tmp"] + objs + ["-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(lib + ".tmp", lib)
    return lib


def _device_object(obj):
    """Extract the gfx950 code object of a compiled .hip object; returns
    (path, cleanup paths), or None when the LLVM tools are missing."""
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-objdump")):
        return None
    subprocess.check_call([os.path.join(llvm, "llvm-objdump"), "--offloading", obj], stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL)
    co = obj + ".0.hipv4-amdgcn-amd-amdhsa--" + ARCH
    return co, (co, obj + ".0.host-x86_64-unknown-linux-gnu-")


def loop_spill_stores(obj, kernel):
    """scratch_store instructions of `kernel` after its first s_sleep (the
    persistent loop's wait): 0 when the kernel spills only in its prologue,
    None when the LLVM tools are missing or the code object holds no such
    kernel (or it has no s_sleep: then the loop cannot be located)."""
    d = _device_object(obj)
    if d is None:
        return None
    co, tmp = d
    try:
        dis = subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", co], text=True)
    finally:
        for f in tmp:
            if os.path.exists(f):
                os.remove(f)
    lines, inside = [], False
    for ln in dis.splitlines():
        if ln.endswith(">:") and " <" in ln:
            if inside:
                break
            inside = ln.split(" <", 1)[1][:-2] == kernel
            continue
        if inside:
            lines.append(ln)
    first = next((i for i, ln in enumerate(lines) if "s_sleep" in ln), None)
    if not lines or first is None:
        return None
    return sum("scratch_store" in ln for ln in lines[first:])


def kernel_vgprs(obj, kernel):
    """VGPR count of `kernel` in a compiled .hip object (its gfx950 code
    object's metadata), or None when the LLVM tools are missing."""
    import re
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-readelf")):
        return None
    subprocess.check_call([os.path.join(llvm, "llvm-objdump"), "--offloading", obj], stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL)
    co = obj + ".0.hipv4-amdgcn-amd-amdhsa--" + ARCH
    host = obj + ".0.host-x86_64-unknown-linux-gnu-"
    try:
        notes = subprocess.check_output([os.path.join(llvm, "llvm-readelf"), "--notes", co], text=True)
    finally:
        for f in (co, host):
            if os.path.exists(f):
                os.remove(f)
    i = notes.find(".name:           " + kernel)
    if i < 0:
        return None
    j = notes.find("\n  - .", i)   # the kernel's metadata entry: from its "- ." line to the next one
    m = re.search(r"\.vgpr_count:\s*(\d+)", notes[notes.rfind("- .", 0, i):j if j > 0 else len(notes)])
    return int(m.group(1)) if m else None


# k_tile_persist's scout wave stopped ~0.7 ms into every run of the builds
# that spill VGPRs inside the persistent loop (round 4: every 256-VGPR build,
# profiles/r04_tile_scout_vgpr_ab.txt; round 5: an inlined scout stops too,
# while a 256-VGPR build that spills only in its prologue runs clean,
# profiles/r05_scout_stop_cause.txt) -- refuse such a build
TILE_KERNEL = "_Z14k_tile_persist18fd_amd_tile_args_t"


def build_diag(force=False, verbose=False):
    """The diagnostics library (FD_AMD_DIAG): tools load it through FD_AMD_LIB."""
    if not force and not _stale(LIB_DIAG, [os.path.join(CSRC, s) for s in SOURCES + HEADERS]):
        return LIB_DIAG
    return build_engine(force=True, verbose=verbose, out=LIB_DIAG, defines=("FD_AMD_DIAG",))


def build_oracle(verbose=False):
    od = os.path.join(ROOT, "oracle")
    out = subprocess.DEVNULL if not verbose else None
    subprocess.check_call(["make", "-C", od, "-j8", "all"], stdout=out)
    if os.path.isdir("/root/reference/src"):
        subprocess.check_call(["make", "-C", od, "-j8", "ref", "tools"], stdout=out)


def build_clients(verbose=False):
    """Plain-C callers of the boundary (gcc, include/*.h only, linked against
    the built library): tests/c/dropin_client."""
    src = os.path.join(ROOT, "tests", "c", "dropin_client.c")
    exe = os.path.join(ROOT, "tests", "c", "dropin_client")
    cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src,
           "-L", os.path.join(ROOT, "firedancer_amd"), "-lfd_ed25519_amd",
           "-Wl,-rpath,$ORIGIN/../../firedancer_amd", "-o", exe]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return exe


def build(force=False, verbose=False):
    build_oracle(verbose)
    so = build_engine(force, verbose)
    build_clients(verbose)
    return so


if __name__ == "__main__":
    # python -m firedancer_amd.build [--force] [--variant OUT.so DEF1,DEF2]  (A/B experiment builds)
    if "--diag" in sys.argv:
        print(build_diag(force="--force" in sys.argv, verbose=True))
    elif "--variant" in sys.argv:
        k = sys.argv.index("--variant")
        out, defs = sys.argv[k + 1], [d for d in sys.argv[k + 2].split(",") if d]
        print(build_engine(force=True, verbose=True, out=os.path.abspath(out), defines=defs,
                           vgpr_guard="--no-vgpr-guard" not in sys.argv))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
