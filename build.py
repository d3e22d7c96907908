#!/usr/bin/env python3
"""Native build driver for brpc_amd.

Generates ``build/build.ninja`` and runs ninja.  Host C++ is compiled with g++
(C++17), device code (``*.hip``) with ``hipcc --offload-arch=gfx950``.  All
artefacts land in-tree so that they travel with the repository snapshot to the
GPU box:

  brpc_amd/lib/libmrpc.so        core runtime (fiber, var, net, rpc, gpu, ...)
  brpc_amd/_native*.so           pybind11 bindings used by python / bench.py
  build/bin/mrpc_protoc          .proto -> C++ generator (bootstrap)
  build/bin/mrpc_unittests       C++ unit tests (driven from pytest)
  build/bin/rpc_press, ...       tools and examples

Usage: python build.py [-j N] [--clean] [--debug] [--asan]
"""
import argparse
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "brpc_amd")
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build")
GEN = os.path.join(BUILD, "gen")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]

# Directories whose sources form the bootstrap library used by mrpc_protoc.
BOOT_DIRS = ["base", "pb"]
# Protos that also get generated mcpack codecs (mrpc_protoc --mcpack_out),
# compiled into libmrpc: the mcpack/ubrpc/nshead_mcpack services' messages.
MCPACK_PROTOS = ["echo", "test_services"]
# Directories excluded from libmrpc.
NON_LIB_DIRS = {"tools", "python", "tests", "examples", "heapprof"}


def rel(p):
    return os.path.relpath(p, BUILD)


def list_sources(subdirs=None, exts=(".cc",)):
    out = []
    for d in sorted(os.listdir(CSRC)):
        full = os.path.join(CSRC, d)
        if not os.path.isdir(full):
            continue
        if subdirs is not None and d not in subdirs:
            continue
        if subdirs is None and d in NON_LIB_DIRS:
            continue
        for ext in exts:
            out += sorted(glob.glob(os.path.join(full, "**", "*" + ext), recursive=True))
    return out


def obj_of(src, suffix=".o"):
    r = os.path.relpath(src, ROOT)
    return os.path.join(BUILD, "obj", r + suffix)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=int(os.environ.get("MAX_JOBS", os.cpu_count() or 8)))
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-only ASan build (never on GPU code)")
    ap.add_argument("--tsan", action="store_true", help="host-only TSan build")
    ap.add_argument("--no-hip", action="store_true", help="skip device code (CPU-only box)")
    ap.add_argument("targets", nargs="*")
    a = ap.parse_args()
    if a.clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.join(PKG, "lib"), exist_ok=True)

    opt = "-O0 -g" if a.debug else "-O2 -g1"
    san = ""
    if a.asan:
        san = "-fsanitize=address -fno-omit-frame-pointer"
    elif a.tsan:
        san = "-fsanitize=thread"
    pyinc = sysconfig.get_paths()["include"]
    import pybind11  # noqa: E402
    pybind_inc = pybind11.get_include()
    ext_suffix = sysconfig.get_config_var("EXT_SUFFIX")

    # TLS descriptors: thread-locals of the dlopen'ed libmrpc (fiber worker
    # state, pool caches, var agents) resolve through _dl_tlsdesc_dynamic's
    # register-preserving fast path instead of a PLT call into
    # __tls_get_addr (17% of a device-codec leg's host samples). initial-exec
    # is not an option: torch's libraries leave no static TLS surplus
    tls = "" if san else "-mtls-dialect=gnu2"
    cxxflags = (f"-std=c++17 {opt} {san} {tls} -fPIC -pthread -march=x86-64-v2 -mpclmul "
                f"-Wall -Wno-unused-function -Wno-invalid-offsetof -Wno-unused-variable "
                f"-Wno-sign-compare -Wno-class-memaccess -Wno-unused-but-set-variable -Wno-unused-result "
                f"-D__HIP_PLATFORM_AMD__ -DMRPC_GPU_ARCH=\\\"{ARCH}\\\" "
                f"-I{rel(CSRC)} -I{rel(GEN)} -isystem {ROCM}/include")
    hipflags = (f"-std=c++17 -O3 -g1 -fPIC --offload-arch={ARCH} -munsafe-fp-atomics "
                f"-I{rel(CSRC)} -I{rel(GEN)}")
    ldlibs = f"-L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lamdhip64 -lssl -lcrypto -lz -ldl -lpthread -lrt"

    boot_srcs = list_sources(BOOT_DIRS)
    lib_srcs = list_sources(None)
    hip_srcs = [] if a.no_hip else list_sources(None, exts=(".hip",))
    protos = sorted(glob.glob(os.path.join(PKG, "proto", "*.proto")))
    gen_ccs = []
    gen_hs = []
    for p in protos:
        b = os.path.splitext(os.path.basename(p))[0]
        gen_ccs.append(os.path.join(GEN, "mrpc", "proto", b + ".pb.cc"))
        gen_hs.append(os.path.join(GEN, "mrpc", "proto", b + ".pb.h"))

    L = []
    w = L.append
    w(f"cxx = g++\nhipcc = {ROCM}/bin/hipcc\n")
    w(f"cxxflags = {cxxflags}\nhipflags = {hipflags}\nldlibs = {ldlibs}\n")
    w("rule cxx\n  command = $cxx $cxxflags $extra -MMD -MF $out.d -c $in -o $out\n"
      "  depfile = $out.d\n  deps = gcc\n  description = CXX $in\n")
    w("rule hip\n  command = $hipcc $hipflags -MMD -MF $out.d -c $in -o $out\n"
      "  depfile = $out.d\n  deps = gcc\n  description = HIP $in\n")
    w("rule ar\n  command = rm -f $out && ar rcs $out $in\n  description = AR $out\n")
    w(f"rule solink\n  command = $cxx -shared {san} -o $out $in $extra $ldlibs\n  description = SO $out\n")
    w(f"rule link\n  command = $cxx {san} -o $out $in $extra $ldlibs\n  description = LINK $out\n")
    w("rule protoc\n  command = $protoc --cpp_out=$gendir --proto_path=$protodir $in\n"
      "  description = PROTOC $in\n")

    def cxx(src, extra="", implicit=()):
        o = obj_of(src)
        imp = (" | " + " ".join(x if x == "gen_headers" else rel(x) for x in implicit)) if implicit else ""
        w(f"build {rel(o)}: cxx {rel(src)}{imp}\n" + (f"  extra = {extra}\n" if extra else ""))
        return o

    boot_objs = [cxx(s) for s in boot_srcs]
    boot_lib = os.path.join(BUILD, "libmrpc_boot.a")
    w(f"build {rel(boot_lib)}: ar {' '.join(rel(o) for o in boot_objs)}\n")
    protoc = os.path.join(BUILD, "bin", "mrpc_protoc")
    protoc_main = cxx(os.path.join(CSRC, "tools", "protoc_main.cc"))
    w(f"build {rel(protoc)}: link {rel(protoc_main)} {rel(boot_lib)}\n")
    for p, cc, h in zip(protos, gen_ccs, gen_hs):
        w(f"build {rel(cc)} {rel(h)}: protoc {rel(p)} | {rel(protoc)}\n"
          f"  protoc = {rel(protoc)}\n  gendir = {rel(os.path.join(GEN, 'mrpc', 'proto'))}\n"
          f"  protodir = {rel(os.path.join(PKG, 'proto'))}\n")
    w("rule protoc_mcpack\n  command = $protoc --mcpack_out=$gendir --proto_path=$protodir $in\n"
      "  description = PROTOC-MCPACK $in\n")
    for p in protos:
        b = os.path.splitext(os.path.basename(p))[0]
        if b not in MCPACK_PROTOS:
            continue
        mc = os.path.join(GEN, "mrpc", "proto", b + ".pb.mcpack.cc")
        w(f"build {rel(mc)}: protoc_mcpack {rel(p)} | {rel(protoc)}\n"
          f"  protoc = {rel(protoc)}\n  gendir = {rel(os.path.join(GEN, 'mrpc', 'proto'))}\n"
          f"  protodir = {rel(os.path.join(PKG, 'proto'))}\n")
        gen_ccs.append(mc)
    w(f"build gen_headers: phony {' '.join(rel(h) for h in gen_hs)}\n")

    lib_objs = []
    for s in lib_srcs:
        if os.path.relpath(s, CSRC).split(os.sep)[0] in BOOT_DIRS:
            lib_objs.append(obj_of(s))
        else:
            lib_objs.append(cxx(s, implicit=["gen_headers"]))
    for cc in gen_ccs:
        lib_objs.append(cxx(cc, implicit=["gen_headers"]))
    for s in hip_srcs:
        o = obj_of(s)
        w(f"build {rel(o)}: hip {rel(s)} | gen_headers\n")
        lib_objs.append(o)
    libso = os.path.join(PKG, "lib", "libmrpc.so")
    w(f"build {rel(libso)}: solink {' '.join(rel(o) for o in lib_objs)}\n")

    rpath = "-Wl,-rpath,'$$ORIGIN/../../brpc_amd/lib' -Wl,-rpath,'$$ORIGIN/lib'"
    linkmrpc = f"-L{rel(os.path.join(PKG, 'lib'))} -lmrpc {rpath}"

    # python module
    py_srcs = sorted(glob.glob(os.path.join(CSRC, "python", "*.cc")))
    py_objs = [cxx(s, extra=f"-isystem {pybind_inc} -isystem {pyinc} -fvisibility=hidden",
                   implicit=["gen_headers"]) for s in py_srcs]
    pymod = os.path.join(PKG, "_native" + ext_suffix)
    w(f"build {rel(pymod)}: solink {' '.join(rel(o) for o in py_objs)} | {rel(libso)}\n"
      f"  extra = {linkmrpc}\n")

    # unit tests
    ut_srcs = sorted(glob.glob(os.path.join(CSRC, "tests", "*.cc")))
    ut_objs = [cxx(s, implicit=["gen_headers"]) for s in ut_srcs]
    bins = []
    if ut_objs:
        ut = os.path.join(BUILD, "bin", "mrpc_unittests")
        w(f"build {rel(ut)}: link {' '.join(rel(o) for o in ut_objs)} | {rel(libso)}\n  extra = {linkmrpc}\n")
        bins.append(ut)
    # stub shared libraries the unit tests dlopen (tests/stub/<name>.cc ->
    # build/lib/lib<name>.so), e.g. the fake verbs library of RdmaVerbs.*
    for s in sorted(glob.glob(os.path.join(CSRC, "tests", "stub", "*.cc"))):
        name = os.path.splitext(os.path.basename(s))[0]
        o = cxx(s, extra="-fvisibility=hidden")
        so = os.path.join(BUILD, "lib", "lib%s.so" % name)
        w(f"build {rel(so)}: solink {rel(o)}\n  ldlibs = -lpthread\n")
        bins.append(so)
    # tools and examples: every tools/<name>.cc except protoc_main, examples/<name>/*.cc
    for s in sorted(glob.glob(os.path.join(CSRC, "tools", "*.cc"))):
        name = os.path.splitext(os.path.basename(s))[0]
        if name == "protoc_main":
            continue
        o = cxx(s, implicit=["gen_headers"])
        b = os.path.join(BUILD, "bin", name)
        w(f"build {rel(b)}: link {rel(o)} | {rel(libso)}\n  extra = {linkmrpc}\n")
        bins.append(b)
    for d in sorted(glob.glob(os.path.join(CSRC, "examples", "*"))):
        if not os.path.isdir(d):
            continue
        for s in sorted(glob.glob(os.path.join(d, "*.cc"))):
            name = os.path.basename(d) + "_" + os.path.splitext(os.path.basename(s))[0]
            o = cxx(s, implicit=["gen_headers"])
            b = os.path.join(BUILD, "bin", name)
            w(f"build {rel(b)}: link {rel(o)} | {rel(libso)}\n  extra = {linkmrpc}\n")
            bins.append(b)
    # sampling heap profiler: never part of libmrpc (it interposes malloc);
    # linked into heapprof_demo and shipped as an LD_PRELOAD library
    hp = os.path.join(CSRC, "heapprof", "heapprof.cc")
    if os.path.exists(hp):
        hp_o = cxx(hp)
        hp_so = os.path.join(PKG, "lib", "libmrpc_heapprof.so")
        w(f"build {rel(hp_so)}: solink {rel(hp_o)}\n  ldlibs = -ldl -lpthread\n")
        d_o = cxx(os.path.join(CSRC, "heapprof", "heapprof_demo.cc"), implicit=["gen_headers"])
        b = os.path.join(BUILD, "bin", "heapprof_demo")
        w(f"build {rel(b)}: link {rel(d_o)} {rel(hp_o)} | {rel(libso)}\n  extra = {linkmrpc} -rdynamic\n")
        bins += [hp_so, b]
    w(f"build all: phony {rel(libso)} {rel(pymod)} {' '.join(rel(b) for b in bins)}\n")
    w("default all\n")
    with open(os.path.join(BUILD, "build.ninja"), "w") as f:
        f.write("\n".join(L))
    cmd = ["ninja", "-C", BUILD, f"-j{a.j}"] + a.targets
    r = subprocess.run(cmd)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
