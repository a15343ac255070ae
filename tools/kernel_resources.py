"""Register / LDS / scratch footprint of the kernels in a hipcc object (gfx950 code-object notes).

    python tools/kernel_resources.py [object.o] [kernel-name-regex]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
KEYS = ("name", "vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "private_segment_fixed_size", "group_segment_fixed_size")


def notes(obj):
    with tempfile.TemporaryDirectory() as t:
        fat, co = os.path.join(t, "fat.bin"), os.path.join(t, "k.co")
        # (on a copy: llvm-objcopy with no output file rewrites its input, which would touch the object's mtime)
        src = os.path.join(t, "obj.o")
        shutil.copyfile(obj, src)
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", src], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{B}/llvm-readobj", "--notes", co], check=True, capture_output=True, text=True).stdout


def kernels(text):
    """One dict per kernel: the metadata block of each `- .args:` entry."""
    out, cur = [], None
    for line in text.splitlines():
        if re.match(r"^  - \.", line):  # a new entry of amdhsa.kernels
            if cur:
                out.append(cur)
            cur = {}
        m = re.match(r"^(?:  - |    )\.(\w+):\s*(\S+)\s*$", line)
        if cur is not None and m and m.group(1) in KEYS and m.group(1) not in cur:
            cur[m.group(1)] = m.group(2)
    if cur:
        out.append(cur)
    return out


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else "jsraytracer_amd/_build/render.o"
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    ks = kernels(notes(obj))
    names = subprocess.run(["c++filt"], input="\n".join(d.get("name", "?") for d in ks), capture_output=True,
                           text=True).stdout.splitlines()
    for d, name in zip(ks, names):
        name = name.replace("jsrt::", "").split("(")[0]
        if not pat.search(name):
            continue
        print(f"{name[:60]:60s} vgpr {d.get('vgpr_count', '-'):>4} agpr {d.get('agpr_count', '-'):>3} "
              f"sgpr {d.get('sgpr_count', '-'):>3} spill {d.get('vgpr_spill_count', '-'):>3} "
              f"scratch {d.get('private_segment_fixed_size', '-'):>5} lds {d.get('group_segment_fixed_size', '-')}")


if __name__ == "__main__":
    main()
