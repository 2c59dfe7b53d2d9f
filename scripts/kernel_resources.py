"""Register / scratch / LDS use of the gfx950 kernels in libspmcts.so (from the code object's
metadata notes): extracts the offload bundle with llvm-objdump and reads llvm-readelf --notes.

    python scripts/kernel_resources.py [regex] [path/to/libspmcts.so]
"""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(so):
    d = tempfile.mkdtemp(prefix="spmcts_co_")
    try:
        x = os.path.join(d, "x.so")
        shutil.copy(so, x)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", x], cwd=d, check=True, capture_output=True)
        out = []
        for f in sorted(glob.glob(os.path.join(d, "x.so.*gfx950*"))):
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f], check=True, capture_output=True,
                                   text=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk)
                if not name:
                    continue

                def num(key):
                    m = re.search(r"\." + key + r":\s+(\d+)", blk)
                    return int(m.group(1)) if m else None

                out.append(dict(name=name.group(1), agpr=int(blk.split("\n")[0].strip(": ")), vgpr=num("vgpr_count"),
                                spill=num("vgpr_spill_count"), scratch=num("private_segment_fixed_size"),
                                lds=num("group_segment_fixed_size")))
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
    so = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                             "self_play_reinforcement_learning_amd", "libspmcts.so")
    for k in kernels(so):
        if pat.search(k["name"]):
            print(f"{k['name'][:110]:110s} vgpr {k['vgpr']:3d} agpr {k['agpr']:3d} spill {k['spill']:4d} "
                  f"scratch {k['scratch']:4d} lds {k['lds']}")


if __name__ == "__main__":
    main()
