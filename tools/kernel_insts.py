"""Static instruction counts of the kernels in a hipcc object (gfx950 disassembly), per class.

    python tools/kernel_insts.py [object.o] [kernel-name-regex]

A quick A/B aid next to kernel_resources.py: how many VALU f64 / f32 / int / SALU / memory / branch
instructions a kernel's code holds (static, not executed counts).
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def disasm(obj):
    with tempfile.TemporaryDirectory() as t:
        fat, co = os.path.join(t, "fat.bin"), os.path.join(t, "k.co")
        # (on a copy: llvm-objcopy with no output file rewrites its input, which would touch the object's mtime)
        src = os.path.join(t, "obj.o")
        shutil.copyfile(obj, src)
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", src], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{B}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                              text=True).stdout


CLASSES = [("cvt", re.compile(r"^v_cvt")), ("f64", re.compile(r"^v_\w*_f64")), ("f32", re.compile(r"^v_\w*_f32")),
           ("valu", re.compile(r"^v_")),
           ("salu", re.compile(r"^s_(?!load|buffer|waitcnt|cbranch|branch|endpgm|barrier|nop|sleep|setprio)")),
           ("smem", re.compile(r"^s_(load|buffer)")), ("vmem", re.compile(r"^(global|buffer|flat|scratch)_")),
           ("lds", re.compile(r"^ds_")), ("branch", re.compile(r"^s_(cbranch|branch)")),
           ("wait", re.compile(r"^s_waitcnt"))]


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else "jsraytracer_amd/_build/render_pf0.o"
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    text = disasm(obj)
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith(";"):
            continue
        funcs[cur].append(s.split()[0])
    names = list(funcs)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    for raw, name in zip(names, dem):
        name = name.replace("jsrt::", "").split("(")[0]
        if not pat.search(name) or not funcs[raw]:
            continue
        counts = {c: 0 for c, _ in CLASSES}
        for op in funcs[raw]:
            for c, rx in CLASSES:
                if rx.match(op):
                    counts[c] += 1
                    break
        print(f"{name[:48]:48s} total {len(funcs[raw]):6d} " + " ".join(f"{c} {n:5d}" for c, n in counts.items()))


if __name__ == "__main__":
    main()
