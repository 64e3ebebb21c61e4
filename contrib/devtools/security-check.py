#!/usr/bin/env python3
"""Check that ELF executables and libraries were built with the hardening the release needs:

* PIE: the executable is position independent (ET_DYN with an interpreter);
* NX: the stack (PT_GNU_STACK) is not executable;
* RELRO: a PT_GNU_RELRO segment and immediate binding (DT_FLAGS BIND_NOW or DT_FLAGS_1 NOW), so
  the GOT is read-only after start-up;
* Canary: the stack protector is linked in (a dynamic reference to __stack_chk_fail).

Parity: reference contrib/devtools/security-check.py (the same four ELF checks; it shells out to
readelf, this one reads the ELF structures itself). Usage: security-check.py FILE... ; prints the
failed checks per file and exits 1 if any failed.
"""
import struct
import sys

ET_DYN = 3
PT_INTERP, PT_GNU_STACK, PT_GNU_RELRO, PT_DYNAMIC = 3, 0x6474E551, 0x6474E552, 2
PF_X = 1
DT_NULL, DT_FLAGS, DT_FLAGS_1 = 0, 30, 0x6FFFFFFB
DF_BIND_NOW, DF_1_NOW, DF_1_PIE = 0x8, 0x1, 0x08000000
SHT_DYNSYM = 11


class Elf:
    def __init__(self, path):
        with open(path, "rb") as f:
            self.data = f.read()
        d = self.data
        if d[:4] != b"\x7fELF" or d[4] != 2 or d[5] != 1:
            raise ValueError(f"{path}: not a 64-bit little-endian ELF file")
        (self.type, _, _, _, self.phoff, self.shoff, _, _, self.phentsize, self.phnum, self.shentsize, self.shnum,
         self.shstrndx) = struct.unpack_from("<HHIQQQIHHHHHH", d, 16)
        self.phdrs = []
        for i in range(self.phnum):
            p_type, p_flags, p_offset, p_vaddr, _, p_filesz, _, _ = struct.unpack_from(
                "<IIQQQQQQ", d, self.phoff + i * self.phentsize)
            self.phdrs.append((p_type, p_flags, p_offset, p_vaddr, p_filesz))
        self.shdrs = []
        for i in range(self.shnum):
            (sh_name, sh_type, _, sh_addr, sh_offset, sh_size, sh_link, _, _, sh_entsize) = struct.unpack_from(
                "<IIQQQQIIQQ", d, self.shoff + i * self.shentsize)
            self.shdrs.append((sh_name, sh_type, sh_addr, sh_offset, sh_size, sh_link, sh_entsize))

    def segments(self, kind):
        return [p for p in self.phdrs if p[0] == kind]

    def dynamic(self):
        out = {}
        for p in self.segments(PT_DYNAMIC):
            off, end = p[2], p[2] + p[4]
            while off + 16 <= end:
                tag, val = struct.unpack_from("<qQ", self.data, off)
                if tag == DT_NULL:
                    break
                out.setdefault(tag, val)
                off += 16
        return out

    def dynamic_symbols(self):
        names = set()
        for (_, sh_type, _, off, size, link, entsize) in self.shdrs:
            if sh_type != SHT_DYNSYM or entsize == 0:
                continue
            stroff = self.shdrs[link][3]
            for i in range(size // entsize):
                st_name = struct.unpack_from("<I", self.data, off + i * entsize)[0]
                end = self.data.index(b"\0", stroff + st_name)
                names.add(self.data[stroff + st_name:end].decode(errors="replace"))
        return names


def check(path):
    e = Elf(path)
    dyn = e.dynamic()
    executable = bool(e.segments(PT_INTERP))
    failed = []
    if executable and not (e.type == ET_DYN or dyn.get(DT_FLAGS_1, 0) & DF_1_PIE):
        failed.append("PIE")
    stack = e.segments(PT_GNU_STACK)
    if not stack or stack[0][1] & PF_X:
        failed.append("NX")
    bind_now = (dyn.get(DT_FLAGS, 0) & DF_BIND_NOW) or (dyn.get(DT_FLAGS_1, 0) & DF_1_NOW)
    if not e.segments(PT_GNU_RELRO) or not bind_now:
        failed.append("RELRO")
    if "__stack_chk_fail" not in e.dynamic_symbols():
        failed.append("Canary")
    return failed


def main(argv):
    status = 0
    for path in argv:
        try:
            failed = check(path)
        except (OSError, ValueError) as err:
            print(f"{path}: cannot check: {err}")
            status = 1
            continue
        if failed:
            print(f"{path}: failed {' '.join(failed)}")
            status = 1
    return status


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
