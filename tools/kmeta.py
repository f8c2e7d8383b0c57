"""Register / spill metadata of the library's gfx950 kernels (from the built kernels.hip.o).

    python tools/kmeta.py [substring ...]      # kernels whose mangled name contains any substring
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "distributed_inference_demo_amd", "build", "kernels.hip.o")
LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", OBJ], cwd=os.path.dirname(OBJ), check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    co = OBJ + ".0.hipv4-amdgcn-amd-amdhsa--gfx950"
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    for f in (co, OBJ + ".0.host-x86_64-unknown-linux-gnu-"):
        if os.path.exists(f):
            os.remove(f)
    pats = sys.argv[1:]
    cur = None
    rows = []
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|vgpr_spill_count|private_segment_fixed_size|agpr_count):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        if pats and not any(p in r["name"] for p in pats):
            continue
        print(f"{r['name'][:90]:90s} vgpr {r.get('vgpr_count', '?'):>4s} agpr {r.get('agpr_count', '?'):>4s} "
              f"spill {r.get('vgpr_spill_count', '?'):>4s} scratch {r.get('private_segment_fixed_size', '?')}")


if __name__ == "__main__":
    main()
