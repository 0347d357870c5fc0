"""Check, on the built library's machine code, that the seeding kernel's
hand-issued claim atomic is not read before its wait.

seed_wp_kernel claims reads with one `global_atomic_add ... off sc0` per wave,
issued from inline asm (smem_kernels.hip, WP_ISSUE, OPT bit 8) and read at the
top of the next iteration, after the iteration's `s_waitcnt vmcnt(0)`.  LLVM
does not track the VMEM result of an inline-asm block, so nothing but the code
the compiler happened to emit keeps a copy or spill of the destination VGPR
from being read before the atomic has returned.  This walks
every control-flow path from each such atomic in the default kernel's code
object and fails if the destination register is read or written by any
instruction before an `s_waitcnt` whose vmcnt is 0 on that path (branches are
followed to both successors; a call or return before the wait also fails).

    python tools/check_claim_wait.py [libsmemgpu.so]

tests/test_claim_asm.py runs it on the library the tests load.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
# the product default: seed_wp_kernel<24, 18, 1, 4> (every OPT bit)
DEFAULT_KERNEL = "_ZN4smem14seed_wp_kernelILi24ELi18ELi1ELi4ELb0ELb0ELb0ELi15EEEvNS_10SeedParamsE"

_INSN = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<(\S+?)\+0x([0-9a-f]+)>")
_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def code_objects(lib: str, workdir: str) -> list[str]:
    """Every gfx950 code object in the library's .hip_fatbin section (one
    clang offload bundle per HIP source, compressed or not)."""
    fb = os.path.join(workdir, "fatbin.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
    data = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(rb"CCOB|__CLANG_OFFLOAD_BUNDLE__", data) if m.start() % 4096 == 0]
    out = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        if data[s:s + 4] == b"CCOB":  # compressed bundle: its header's total size (v3: u64 at +8)
            ver = int.from_bytes(data[s + 4:s + 6], "little")
            e = s + int.from_bytes(data[s + 8:s + (16 if ver >= 3 else 12)], "little")
        part = os.path.join(workdir, f"b{i}.bin")
        with open(part, "wb") as fh:
            fh.write(data[s:e])
        co = os.path.join(workdir, f"b{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            f"--targets={TARGET}", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def disassemble(co: str, symbol: str) -> list[tuple[int, str, str]] | None:
    """(address, mnemonic, operands) of every instruction of `symbol`, or None."""
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--disassemble-symbols={symbol}", co],
                         capture_output=True, text=True, check=True).stdout
    if f"<{symbol}>:" not in txt:
        return None
    insns = []
    for line in txt.splitlines():
        m = _INSN.match(line)
        if m:
            insns.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return insns


def _regs(ops: str) -> set[int]:
    r = set()
    for m in _VREG.finditer(ops):
        if m.group(1) is not None:
            r.add(int(m.group(1)))
        else:
            r.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return r


def _waits_vm0(mn: str, ops: str) -> bool:
    if mn != "s_waitcnt":
        return False
    m = re.search(r"vmcnt\((\d+)\)", ops)
    return m is not None and int(m.group(1)) == 0


def check(insns: list[tuple[int, str, str]], base: int | None = None) -> tuple[int, list[str]]:
    """Returns (hand-issued claim atomics found, violations)."""
    addr_ix = {a: i for i, (a, _, _) in enumerate(insns)}
    if base is None:
        base = insns[0][0]
    atomics = [i for i, (_, mn, ops) in enumerate(insns)
               if mn == "global_atomic_add" and ops.rstrip().endswith("off sc0")]
    bad = []
    for ai in atomics:
        dst = int(re.match(r"v(\d+)", insns[ai][2]).group(1))
        seen = set()
        todo = [ai + 1]
        while todo:
            i = todo.pop()
            while i < len(insns) and i not in seen:
                seen.add(i)
                a, mn, ops = insns[i]
                if _waits_vm0(mn, ops):
                    break
                if dst in _regs(ops):
                    bad.append(f"v{dst} (claim at {insns[ai][0]:#x}) used at {a:#x}: {mn} {ops}")
                    break
                if mn in ("s_endpgm",):
                    break
                if mn.startswith("s_swappc") or mn.startswith("s_setpc") or mn.startswith("s_call"):
                    bad.append(f"call/return at {a:#x} before the wait for v{dst}")
                    break
                if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
                    t = _TARGET.search(ops)
                    # the disassembler prints the target as <symbol+0xoff> in the operand comment;
                    # fall back to the immediate (dwords after the branch)
                    tgt = None
                    if t is not None:
                        tgt = addr_ix.get(base + int(t.group(2), 16))
                    if tgt is None:
                        m = re.match(r"(-?\d+)", ops)
                        if m:
                            tgt = addr_ix.get(a + 4 + 4 * int(m.group(1)))
                    if tgt is None:
                        bad.append(f"unresolved branch at {a:#x}: {mn} {ops}")
                        break
                    todo.append(tgt)
                    if mn.startswith("s_branch"):
                        break
                i += 1
    return len(atomics), bad


def run(lib: str, symbol: str = DEFAULT_KERNEL) -> tuple[int, list[str]]:
    with tempfile.TemporaryDirectory() as td:
        for co in code_objects(lib, td):
            insns = disassemble(co, symbol)
            if insns:
                return check(insns)
    raise RuntimeError(f"{symbol} not found in {lib}")


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bwa-mem-harp2_amd", "lib", "libsmemgpu.so")
    n, bad = run(lib)
    print(f"{n} hand-issued claim atomic(s) in the default seeding kernel; {len(bad)} early use(s)")
    for b in bad:
        print("  " + b)
    sys.exit(1 if bad or n == 0 else 0)
