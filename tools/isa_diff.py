#!/usr/bin/env python3
"""Compare the gfx950 machine code of two builds of the library, kernel by kernel (a refactor that must not change
the product's code: pruned variant macros, moved helpers).

    python tools/isa_diff.py A.so B.so [--show KERNEL]

Extracts the hipv4 gfx950 code object of each library (objcopy + clang-offload-bundler), disassembles it
(llvm-objdump -d), drops addresses / encodings / branch-target labels, and reports the kernels whose instruction
sequences differ, plus kernels present in only one build.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib, tmp):
    """The gfx950 code object of every translation unit (the .hip_fatbin section holds one offload bundle per
    compiled source, concatenated)."""
    fb = os.path.join(tmp, os.path.basename(lib) + ".fatbin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = []
    i = data.find(magic)
    while i >= 0:
        starts.append(i)
        i = data.find(magic, i + 1)
    cos = []
    for n, (a, b) in enumerate(zip(starts, starts[1:] + [len(data)])):
        part = os.path.join(tmp, f"{os.path.basename(lib)}.{n}.bundle")
        co = os.path.join(tmp, f"{os.path.basename(lib)}.{n}.co")
        open(part, "wb").write(data[a:b])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
        cos.append(co)
    return cos


def kernels(cos):
    out = "".join(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--no-leading-addr", co],
                                 capture_output=True, text=True, check=True).stdout for co in cos)
    ks, name = {}, None
    for line in out.splitlines():
        m = re.match(r"^([0-9a-f]+ )?<(.+)>:$", line.strip())
        if m:
            name = m.group(2)
            ks[name] = []
            continue
        if name is None:
            continue
        s = line.split("//")[0].strip()
        if not s or "file format" in s or s.startswith("Disassembly of section"):
            continue
        s = re.sub(r"<[^>]+>", "<L>", s)                  # branch targets by label
        s = re.sub(r"0x[0-9a-f]+", "IMM", s) if s.startswith("s_getpc") else s
        ks[name].append(s)
    return ks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--show", default=None)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        A, B = kernels(code_objects(a.a, tmp)), kernels(code_objects(a.b, tmp))
    only_a, only_b = sorted(set(A) - set(B)), sorted(set(B) - set(A))
    diff = sorted(k for k in set(A) & set(B) if A[k] != B[k])
    same = len(set(A) & set(B)) - len(diff)
    print(f"{same} identical, {len(diff)} differ, {len(only_a)} only in A, {len(only_b)} only in B")
    for k in diff:
        print(f"  differ: {k} ({len(A[k])} vs {len(B[k])} instructions)")
    for k in only_a:
        print(f"  only A: {k}")
    for k in only_b:
        print(f"  only B: {k}")
    if a.show:
        import difflib
        for k in diff:
            if a.show in k:
                sys.stdout.writelines(difflib.unified_diff([x + "\n" for x in A[k]], [x + "\n" for x in B[k]], "A", "B",
                                                           n=2))
    return 1 if (diff or only_a or only_b) else 0


if __name__ == "__main__":
    sys.exit(main())
