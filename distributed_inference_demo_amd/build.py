"""Build libbloomstage.so (gfx950) in-tree with hipcc; no torch extension machinery.

    python -m distributed_inference_demo_amd.build          # incremental
    python -m distributed_inference_demo_amd.build --force
"""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "lib", "libbloomstage.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["kernels.hip", "attn_prefill.hip", "stage.hip", "codec.cpp", "safetensors.cpp"]
# per-source extra flags: the prefill attention keeps its MFMA accumulators in VGPRs (attn_prefill.hip header)
EXTRA = {"attn_prefill.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}
HEADERS = ["common.h", "kernels.h", "attn_merge.h", "safetensors.h"]
STAMP = os.path.join(OBJ, "build_id")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-Wno-unused-result", "-Wno-unused-value", f"-I{os.path.join(ROOT, 'include')}"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def source_hash() -> str:
    """SHA-256 over the library's sources (name + bytes, fixed order): the build provenance stamp
    compiled into bs_build_id() and checked by stage.lib()."""
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "bloomstage.h")]:
        with open(path, "rb") as f:
            h.update(os.path.basename(path).encode() + b"\0" + f.read())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    bid = source_hash()
    old = open(STAMP).read().strip() if os.path.exists(STAMP) else ""
    restamp = old != bid  # only stage.hip carries the stamp
    hdr_t = max([_mtime(os.path.join(CSRC, h)) for h in HEADERS] + [_mtime(os.path.join(ROOT, "include", "bloomstage.h"))])
    jobs = []
    objs = []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        op = os.path.join(OBJ, src + ".o")
        objs.append(op)
        if force or (restamp and src == "stage.hip") or _mtime(op) < max(_mtime(sp), hdr_t):
            flags = list(CFLAGS)
            if src.endswith(".cpp"):
                flags = [f for f in flags if not f.startswith("--offload-arch")] + ["-x", "c++"]
            if src == "stage.hip":
                flags.append(f'-DBS_BUILD_ID="{bid}"')
            flags += EXTRA.get(src, [])
            jobs.append([HIPCC] + flags + ["-c", sp, "-o", op])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        for err in ex.map(run, jobs):
            if err and verbose:
                print(err)
    if jobs or not os.path.exists(LIB) or any(_mtime(o) > _mtime(LIB) for o in objs):
        # -z defs: an unresolved symbol (e.g. a kernel launch stub the host pass dropped) fails the link
        # instead of shipping a library that fails at load time
        run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,-z,defs", "-o", LIB] + objs)
    with open(STAMP, "w") as f:
        f.write(bid)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
