"""Scan the built library's gfx950 code for the wide-store data hazard behind the round-4
RGB warp mismatch.

A VMEM store of more than 8 bytes (buffer/global/flat *_dwordx3 / *_dwordx4) needs one wait
state before another instruction writes the VGPRs that hold its data; without it the store
can pick up the new value when its data read is delayed (memory-pipeline back-pressure), so
the fault is intermittent.  The compiler pads the instructions it generates; it does not pad
around inline asm, so an inline-asm VALU that lands right behind such a store is unchecked.

This tool extracts every gfx950 code object from libkcmc.so's .hip_fatbin section (one
clang offload bundle per source file), disassembles it with llvm-objdump and reports every
wide store whose data VGPRs are written by the very next instruction (zero wait states).

    python tools/debug/store_hazard_scan.py [path/to/libkcmc.so]      (exit 1 on a finding)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
WIDE = re.compile(r"^(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128|format_xyzw?)\b")
VREG = re.compile(r"^v\[(\d+):(\d+)\]$|^v(\d+)$")


def code_objects(lib):
    """(bundle entry id, ELF bytes) of every gfx950 entry of the library's fat binary."""
    with tempfile.TemporaryDirectory() as tmp:
        fat = os.path.join(tmp, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib, "/dev/null"],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        p = pos + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            ident = data[p:p + idlen].decode()
            p += idlen
            if "gfx950" in ident and size:
                out.append((ident, data[pos + off:pos + off + size]))
        pos = data.find(MAGIC, pos + 1)
    return out


def regs(tok):
    m = VREG.match(tok.strip().rstrip(","))
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def scan_text(text):
    """[(function, store line, next line)] for wide stores whose data the next instruction writes."""
    findings, fn = [], "?"
    lines = [l.split(";")[0].strip() for l in text.splitlines()]
    ins = []
    for l in lines:
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", l)
        if m:
            fn = m.group(1)
            continue
        m = re.match(r"^([a-z_][a-z0-9_]*)\s*(.*?)(//.*)?$", l)
        if m and not l.endswith(":") and "_" in m.group(1):
            ins.append((fn, m.group(1), m.group(2)))
    for k, (fn, op, args) in enumerate(ins[:-1]):
        if not WIDE.match(op):
            continue
        toks = [t.strip() for t in args.split(",")]
        data = regs(toks[0]) if op.startswith("buffer_") else regs(toks[1]) if len(toks) > 1 else set()
        nfn, nop, nargs = ins[k + 1]
        if nfn != fn or nop.startswith(("s_", "buffer_store", "global_store", "flat_store", "scratch_store")):
            continue
        dst = regs(nargs.split(",")[0]) if nargs else set()
        if dst & data:
            findings.append((fn, f"{op} {args}", f"{nop} {nargs}"))
    return findings


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(R, "keypoint-consensus-motion-correction_amd", "libkcmc.so")
    total = 0
    n_wide = 0
    with tempfile.TemporaryDirectory() as tmp:
        for k, (ident, elf) in enumerate(code_objects(lib)):
            path = os.path.join(tmp, f"co{k}.elf")
            open(path, "wb").write(elf)
            text = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", path],
                                  check=True, capture_output=True, text=True).stdout
            n_wide += sum(1 for l in text.splitlines() if WIDE.match(l.split(";")[0].strip().split(" ")[0] or "x"))
            for fn, st, nxt in scan_text(text):
                total += 1
                print(f"HAZARD {fn}\n    {st}\n    {nxt}")
    print(f"{n_wide} wide stores scanned, {total} followed by a write of their data registers with no wait state")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
