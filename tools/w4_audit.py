"""Audit of the inline-asm wide-wave GEMM kernels (csrc/gemm_w4.inc) in a built object: the asm fragment
reads are invisible to the compiler's waitcnt pass, so no instruction other than another LDS read may touch
a read's destination VGPRs between the read and the next `s_waitcnt lgkmcnt(0)`; and no scratch (a spill
of an AGPR accumulator written by an asm MFMA would read it before the MFMA's result is ready).

    python tools/w4_audit.py [vit-project_amd/csrc/build/gemm.o] [kernel-name regex, default w4]

Exit status 1 and a report per violation; 0 and a one-line summary per kernel otherwise.
"""
import os, re, subprocess, sys, tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble(obj):
    d = tempfile.mkdtemp()
    fb, dev = os.path.join(d, "fb"), os.path.join(d, "dev.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}", "--unbundle"], check=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", dev], check=True, capture_output=True, text=True).stdout


def audit(text, pat):
    kernels, cur, name = {}, None, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            name = m.group(1)
            cur = kernels.setdefault(name, []) if re.search(pat, name) else None
            continue
        if cur is not None and line.startswith("\t"):
            cur.append(line.split("//")[0].strip())
    bad = 0
    for name, ins in kernels.items():
        pending, nread, nscratch, nviol = set(), 0, 0, 0
        for k, s in enumerate(ins):
            op = s.split(" ")[0]
            if op.startswith("scratch_"):
                nscratch += 1
            if op.startswith("ds_read"):
                dst = s.split(" ", 1)[1].split(",")[0]
                src = s.split(" ", 1)[1].split(",", 1)[1] if "," in s else ""
                if regs(src) & pending:
                    nviol += 1
                    print(f"VIOLATION {name[:70]} #{k}: address of {s!r} is a pending read destination")
                pending |= regs(dst)
                nread += 1
                continue
            if op == "s_waitcnt" and "lgkmcnt(0)" in s:
                pending.clear()
                continue
            touched = regs(s.split(" ", 1)[1]) if " " in s else set()
            if touched & pending:
                nviol += 1
                print(f"VIOLATION {name[:70]} #{k}: {s!r} touches pending read destination(s) "
                      f"{sorted(touched & pending)[:8]}")
        if nscratch:
            print(f"VIOLATION {name[:70]}: {nscratch} scratch instructions")
        bad += nviol + (nscratch > 0)
        print(f"{'ok ' if not (nviol or nscratch) else 'BAD'} {name[:90]}: {len(ins)} instructions, "
              f"{nread} LDS reads, {nviol} hazards, {nscratch} scratch")
    if not kernels:
        print("no kernel matched", pat)
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "vit-project_amd",
                                                               "csrc", "build", "gemm.o")
    sys.exit(audit(disassemble(obj), sys.argv[2] if len(sys.argv) > 2 else r"w4"))
