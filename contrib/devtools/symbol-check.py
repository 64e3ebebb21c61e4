#!/usr/bin/env python3
"""Check that release binaries only depend on what the target systems provide:

* every versioned dynamic symbol needs at most the given glibc / libstdc++ / libgcc versions
  (the ROCm 7 images ship Ubuntu 22.04: glibc 2.35, GLIBCXX 3.4.30);
* every NEEDED library is on the allow-list (the C/C++ runtime, OpenSSL's libcrypto and the
  HIP runtime, which the GPU paths load).

Parity: reference contrib/devtools/symbol-check.py (MAX_VERSIONS and ALLOWED_LIBRARIES checks
over `readelf --dyn-syms` / `readelf -d`). Usage: symbol-check.py FILE... ; exits 1 on any
violation.
"""
import re
import subprocess
import sys

MAX_VERSIONS = {
    "GLIBC": (2, 35),
    "GLIBCXX": (3, 4, 30),
    "CXXABI": (1, 3, 13),
    "GCC": (12, 0, 0),
}
IGNORE_LIBS = {"OPENSSL", "hip"}  # versioned by their own libraries, which the allow-list pins
ALLOWED_LIBRARIES = {
    "libc.so.6", "libm.so.6", "libstdc++.so.6", "libgcc_s.so.1", "libpthread.so.0", "libdl.so.2", "librt.so.1",
    "ld-linux-x86-64.so.2", "libcrypto.so.3", "libamdhip64.so.7",
}
READELF = "readelf"


def versioned_imports(path):
    out = subprocess.run([READELF, "--dyn-syms", "-W", path], capture_output=True, text=True, check=True).stdout
    syms = []
    for line in out.splitlines():
        parts = line.split()
        if len(parts) < 8 or not parts[0].rstrip(":").isdigit():
            continue
        if parts[6] != "UND":  # imports only
            continue
        name = parts[7]
        if "@" in name:
            sym, _, version = name.partition("@")
            syms.append((sym, version.lstrip("@")))
    return syms


def needed_libraries(path):
    out = subprocess.run([READELF, "-d", "-W", path], capture_output=True, text=True, check=True).stdout
    return re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out)


def version_ok(version):
    lib, _, num = version.partition("_")
    if lib in IGNORE_LIBS or not num:
        return True
    if lib not in MAX_VERSIONS:
        return False
    try:
        v = tuple(int(x) for x in num.split("."))
    except ValueError:
        return False
    return v <= MAX_VERSIONS[lib]


def check(path):
    errors = []
    for sym, version in versioned_imports(path):
        if not version_ok(version):
            errors.append(f"symbol {sym} from unsupported version {version}")
    for lib in needed_libraries(path):
        if lib not in ALLOWED_LIBRARIES:
            errors.append(f"NEEDED library {lib} is not allowed")
    return errors


def main(argv):
    status = 0
    for path in argv:
        try:
            errors = check(path)
        except (OSError, subprocess.CalledProcessError) as err:
            print(f"{path}: cannot check: {err}")
            status = 1
            continue
        for e in errors:
            print(f"{path}: {e}")
        if errors:
            status = 1
    return status


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
