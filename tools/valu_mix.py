"""Static VALU instruction mix of one kernel of libo3dx's grid object (packed
f32, f64, transcendental shares), for bench.py's weighted VALU-issue floor.
Usage: python tools/valu_mix.py [mangled-kernel-name] > profiles/r02_valu_mix.json"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "open3d-py-extension_amd", "open3dpypro", "_lib", "obj", "grid.o")
LLVM = "/opt/rocm/lib/llvm/bin"
DEFAULT = "_ZN4o3dx15k_normals_stileILi32ELi2ELi2ELi3ELb0ELb0ELb0EEEvNS_8DenseVoxEiPKfPfPiS5_ii"


def main(name=DEFAULT):
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", OBJ], check=True, capture_output=True)
    dev = OBJ + ".0.hipv4-amdgcn-amd-amdhsa--gfx950"
    try:
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", dev], check=True,
                             capture_output=True, text=True).stdout
    finally:
        for f in (dev, OBJ + ".0.host-x86_64-unknown-linux-gnu-"):
            if os.path.exists(f):
                os.remove(f)
    i = txt.index(name + ">:")
    j = txt.find(">:", i + len(name) + 3)
    ins = [ln.split()[0] for ln in txt[i:j if j > 0 else None].splitlines()
           if re.match(r"\s+(v_|s_|ds_|global_|buffer_)", ln)]
    v = [x for x in ins if x.startswith("v_")]
    out = {"kernel": name, "instructions": len(ins), "valu": len(v),
           "pk": sum(x.startswith("v_pk_") for x in v), "f64": sum(x.endswith("_f64") for x in v),
           "trans": sum(any(t in x for t in ("v_sqrt", "v_rsq", "v_rcp", "v_exp", "v_log", "v_sin", "v_cos"))
                        for x in v),
           "lds": sum(x.startswith("ds_") for x in ins)}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:2])
