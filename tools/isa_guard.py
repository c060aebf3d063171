"""ISA guard for libvge.so's gfx950 code objects (CPU only: no GPU, no compiler run).

Extracts every gfx950 code object from the library's .hip_fatbin section (clang offload bundles), disassembles it with
the ROCm llvm-objdump and reads each kernel's private segment (scratch) size from its AMDGPU metadata note.  Used by
tests/test_isa_guard.py: the hot kernels must carry no FLAT memory instructions (an LDS operand reached through a
generic pointer: the instruction class that can raise a memory violation from an LDS-intended address, DESIGN.md
section 3.2 on the dropped 16x16x32 build's fault) and no scratch.

    python tools/isa_guard.py [libvge.so]   -> one line per kernel: name, scratch bytes/lane, FLAT / scratch ops
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile
from typing import Dict, List

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def fatbin_section(lib: str) -> bytes:
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "fb.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, out], check=True)
        with open(out, "rb") as f:
            return f.read()


def code_objects(lib: str, arch: str = "gfx950") -> List[bytes]:
    """The arch's code objects of every offload bundle in the library (one per HIP translation unit)."""
    data = fatbin_section(lib)
    objs = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if triple.endswith(arch) and size:
                objs.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 24)
    return objs


def kernels(lib: str, arch: str = "gfx950") -> Dict[str, dict]:
    """{mangled kernel name: {scratch, flat, scratch_ops}} over the library's code objects."""
    res: Dict[str, dict] = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(lib, arch)):
            p = os.path.join(td, f"co{k}.elf")
            with open(p, "wb") as f:
                f.write(co)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", p], capture_output=True, text=True,
                                   check=True).stdout
            # the metadata note lists each kernel's .name ... .private_segment_fixed_size (msgpack as YAML text)
            cur = None
            for line in notes.splitlines():
                m = re.match(r"\s*\.name:\s+(\S+)", line)
                if m:
                    cur = m.group(1)
                    res.setdefault(cur, {"scratch": 0, "flat": 0, "scratch_ops": 0})
                m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
                if m and cur:
                    res[cur]["scratch"] = int(m.group(1))
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={arch}", p], capture_output=True, text=True,
                                 check=True).stdout
            sym = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    sym = m.group(1)
                    continue
                if sym in res:
                    s = line.strip()
                    if s.startswith("flat_load") or s.startswith("flat_store") or s.startswith("flat_atomic"):
                        res[sym]["flat"] += 1
                    elif s.startswith("scratch_") or ("buffer_" in s and " off, s[0:3]" in s):
                        res[sym]["scratch_ops"] += 1
    return res


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "video-gen-evals_amd",
                                                              "vge", "libvge.so")
    for name, r in sorted(kernels(lib).items()):
        print(f"{r['scratch']:5d} B/lane  flat {r['flat']:5d}  scratch ops {r['scratch_ops']:4d}  {name}")
