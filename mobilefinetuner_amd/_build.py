"""In-tree native build driver (gfx950 only).

Compiles every HIP kernel (``csrc/kernels/*.hip``) with ``hipcc --offload-arch=gfx950`` and every
host C++ source (``csrc/runtime/*.cpp``, ``csrc/*.cpp``) into ONE python extension
``mobilefinetuner_amd/_C.so`` that links against the HIP runtime bundled with PyTorch-ROCm
(same soname ``libamdhip64.so.7``, so only one HIP runtime is ever loaded in the process).

No hipify, no torch JIT cache: objects live under ``build/`` in the repo and are rebuilt only when
a source or header changed (content hash), so the ``.so`` travels with the repo snapshot to the
GPU box.  Usage::

    python -m mobilefinetuner_amd._build            # build (parallel)
    python -m mobilefinetuner_amd._build --native   # kernels + engine + native CLIs only (no torch import)
    python -m mobilefinetuner_amd._build --clean
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(REPO_DIR, "build", "obj")
OUT_SO = os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("MFT_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch  # noqa: local import keeps `--help` fast
    tdir = os.path.dirname(torch.__file__)
    incs = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    libdir = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, libdir, abi


def _headers_digest() -> str:
    h = hashlib.sha1()
    for p in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


def _sources():
    hip = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    binding = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    return hip, cpp, binding


def _engine_sources():
    """libmft engine (csrc/engine: tensor, allocator, autograd, ops, models, trainer -- no torch) and
    the native CLI mains (csrc/apps)."""
    hip = sorted(glob.glob(os.path.join(CSRC, "engine", "*.hip")))
    cpp = sorted(glob.glob(os.path.join(CSRC, "engine", "*.cpp")))
    apps = sorted(glob.glob(os.path.join(CSRC, "apps", "*.cpp")))
    return hip, cpp, apps


BIN_DIR = os.path.join(PKG_DIR, "bin")
# executable -> (main source, extra defines)
APPS = {
    "gpt2_lora_finetune": ("gpt2_finetune.cpp", []),
    "gpt2_full_finetune": ("gpt2_finetune.cpp", ["-DMFT_FULL_FT=1"]),
    "engine_selftest": ("engine_selftest.cpp", []),
    "eval_ppl": ("eval_ppl.cpp", []),
    "train_lora_gemma": ("train_lora_gemma.cpp", []),
    "eval_mmlu": ("eval_mmlu.cpp", []),
}


def _flags(kind: str, incs, abi):
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}",
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    if kind == "hip":
        # Device code: gfx950 only. -ffp-contract=fast lets hipcc fuse mul+add into v_fma/v_pk_fma.
        return common + [f"--offload-arch={ARCH}", "-ffp-contract=fast", "-munsafe-fp-atomics",
                         "-fgpu-rdc" if False else "-fno-gpu-rdc"]
    py_inc = sysconfig.get_paths()["include"]
    torch_flags = [f"-I{i}" for i in incs] + [f"-I{py_inc}", f"-I{ROCM}/include",
                                             "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                                             "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    if kind == "binding":
        return common + torch_flags
    return common + [f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__=1"]


def _compile_one(src: str, kind: str, flags, hdr_digest: str, verbose: bool, tag: str = ""):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__") + (f"__{tag}" if tag else "")
    obj = os.path.join(BUILD_DIR, rel + ".o")
    stamp = obj + ".sha1"
    with open(src, "rb") as f:
        key = hashlib.sha1(f.read() + hdr_digest.encode() + " ".join(flags).encode()).hexdigest()
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == key:
        return obj, False
    if kind == "hip":
        cmd = [HIPCC, "-x", "hip", *flags, "-c", src, "-o", obj]
    elif kind == "binding":
        cmd = ["g++", *flags, "-c", src, "-o", obj]
    else:
        cmd = ["g++", *flags, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(key)
    return obj, True


def build_native(verbose: bool = False, jobs: int | None = None, abi: int | None = None) -> list:
    """The torch-free part alone: every HIP kernel, the runtime and the libmft engine, linked into the
    native CLIs (mobilefinetuner_amd/bin/).  Imports nothing from torch; the C++ ABI of the objects is
    the one torch was built with (recorded by the last full build, else MFT_CXX11_ABI, default 1) so the
    same objects serve _C.so."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    if abi is None:
        abi = int(os.environ.get("MFT_CXX11_ABI", _recorded_abi()))
    hdr = _headers_digest()
    hip, cpp, _ = _sources()
    jobs = jobs or min(8, max(1, (os.cpu_count() or 4)))
    work = [(s, "hip") for s in hip] + [(s, "cpp") for s in cpp]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = [f.result()[0] for f in [ex.submit(_compile_one, s, k, _flags(k, [], abi), hdr, verbose) for s, k in work]]
    return build_engine(objs_kernels=[o for (s, k), o in zip(work, objs) if k == "hip"],
                        objs_runtime=[o for (s, k), o in zip(work, objs) if k == "cpp"], abi=abi, hdr=hdr,
                        verbose=verbose, jobs=jobs)


def _recorded_abi() -> str:
    try:
        with open(os.path.join(BUILD_DIR, "torch_abi.txt")) as f:
            return f.read().strip() or "1"
    except OSError:
        return "1"


def build(verbose: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    incs, libdir, abi = _torch_paths()
    with open(os.path.join(BUILD_DIR, "torch_abi.txt"), "w") as f:
        f.write(str(abi))
    hdr = _headers_digest()
    hip, cpp, binding = _sources()
    work = [(s, "hip") for s in hip] + [(s, "cpp") for s in cpp] + [(s, "binding") for s in binding]
    jobs = jobs or min(8, max(1, (os.cpu_count() or 4)))
    objs, changed = [], False
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile_one, s, k, _flags(k, incs, abi), hdr, verbose) for s, k in work]
        for f in futs:
            o, c = f.result()
            objs.append(o)
            changed |= c
    if changed or not os.path.exists(OUT_SO):
        tmp = OUT_SO + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp,
               f"-L{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip",
               "-ltorch_hip", "-lamdhip64", f"-L{ROCM}/lib", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{libdir}",
               f"-Wl,-rpath,{ROCM}/lib", "-ldl", "-lpthread"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, OUT_SO)
    build_engine(objs_kernels=[o for (src, k), o in zip(work, objs) if k == "hip"],
                 objs_runtime=[o for (src, k), o in zip(work, objs) if k == "cpp"], abi=abi, hdr=hdr,
                 verbose=verbose, jobs=jobs)
    return OUT_SO


def build_engine(objs_kernels, objs_runtime, abi, hdr, verbose=False, jobs=None) -> list:
    """Compile the torch-free libmft engine and link the native CLIs into mobilefinetuner_amd/bin/
    against the same kernel / runtime objects as _C.so (HIP runtime + RCCL from ROCm; no GEMM library)."""
    os.makedirs(BIN_DIR, exist_ok=True)
    ehip, ecpp, apps = _engine_sources()
    work = [(s, "hip", []) for s in ehip] + [(s, "cpp", []) for s in ecpp]
    app_work = []
    for exe, (main, defs) in APPS.items():
        src = os.path.join(CSRC, "apps", main)
        if os.path.exists(src):
            app_work.append((exe, src, defs))
    jobs = jobs or min(8, max(1, (os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile_one, s, k, _flags(k, [], abi) + d, hdr, verbose) for s, k, d in work]
        app_futs = {exe: ex.submit(_compile_one, src, "cpp", _flags("cpp", [], abi) + defs, hdr, verbose, exe)
                    for exe, src, defs in app_work}
        eobjs = [f.result() for f in futs]
        aobjs = {exe: f.result() for exe, f in app_futs.items()}
    changed = any(c for _, c in eobjs) or any(c for _, c in aobjs.values())
    libs = [o for o, _ in eobjs] + list(objs_kernels) + list(objs_runtime)
    out = []
    for exe, (obj, _) in aobjs.items():
        path = os.path.join(BIN_DIR, exe)
        if changed or not os.path.exists(path) or os.path.getmtime(path) < max(os.path.getmtime(o) for o in libs):
            cmd = [HIPCC, "-fPIC", obj, *libs, "-o", path + ".tmp", f"-L{ROCM}/lib", "-lrccl", "-lamdhip64",
                   "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM}/lib", "-ldl", "-lpthread"]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
            os.replace(path + ".tmp", path)
        out.append(path)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--native", action="store_true", help="the torch-free kernels + engine + CLIs only (no _C.so)")
    a = ap.parse_args(argv)
    if a.clean:
        shutil.rmtree(os.path.join(REPO_DIR, "build"), ignore_errors=True)
        if os.path.exists(OUT_SO):
            os.remove(OUT_SO)
    if a.native:
        print("\n".join(build_native(verbose=a.verbose, jobs=a.jobs)))
        return
    print(build(verbose=a.verbose, jobs=a.jobs))


if __name__ == "__main__":
    main(sys.argv[1:])
