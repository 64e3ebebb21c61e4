#!/usr/bin/env python3
"""Every command-line option the code reads must appear in the -help output of the program
that reads it.

Scans csrc/ for GetArg / GetBoolArg / IsArgSet / GetArgs / SoftSet*Arg / ForceSetArg uses of
"-name" and compares them with the options printed by `bcpd -help`, `bcp-cli -help` and
`bcp-tx -help`. Options that are internal test hooks are listed in UNDOCUMENTED on purpose.

Parity: reference contrib/devtools/check-doc.py (same scan of the sources against the help
strings, with a short allow-list of hidden options). Usage: check-doc.py [REPO_ROOT]; prints
the undocumented options and exits 1 if there are any.

With --reference it also walks contrib/devtools/reference_options.txt (every option the
reference node reads or documents) and reports each one this tree neither reads nor
documents, apart from REFERENCE_NOT_APPLICABLE (the Qt GUI's own switches: this node's GUI is
the browser wallet, see -webgui).
"""
import os
import re
import subprocess
import sys

USE = re.compile(r'(?:GetArg|GetBoolArg|IsArgSet|GetArgs|SoftSetArg|SoftSetBoolArg|ForceSetArg|ClearArg|ParseFeeArg)'
                 r'\(\s*(?:std::string\()?\s*"(-[a-zA-Z0-9][a-zA-Z0-9_.-]*)"')
HELP = re.compile(r"^\s*(-[a-zA-Z0-9][a-zA-Z0-9_.-]*)", re.M)
USAGE = re.compile(r"(?<![\w-])(-[a-zA-Z][a-zA-Z0-9_.-]*)")  # options inlined in a Usage: line
# options the code reads that are deliberately not in -help (test and developer hooks, as the
# reference's -help-debug ones), or set only internally
UNDOCUMENTED = {
    "-gpufaultinjection", "-dropmessagestest", "-fuzzmessagestest", "-mocktime", "-stopafterblockimport",
    "-checkblockindex", "-checkmempool", "-limitfreerelay", "-relaypriority", "-datadir", "-conf", "-help",
    "-version", "-?", "-h", "-regtest", "-testnet", "-fastprune", "-banscore",
    # obsolete options, read only to refuse them or warn (reference init.cpp:1336-1358)
    "-benchmark", "-blockminsize", "-debugnet", "-rpcssl", "-socks", "-tor", "-whitelistalwaysrelay",
}
# reference options with no counterpart here: the Qt wallet's startup switches
REFERENCE_NOT_APPLICABLE = {"-choosedatadir", "-lang", "-min", "-resetguisettings", "-splash", "-uiplatform"}


def used_options(root):
    found = {}
    for d, _, files in os.walk(os.path.join(root, "csrc")):
        if os.sep + "test" in d:
            continue
        for f in files:
            if not f.endswith((".cpp", ".h")):
                continue
            p = os.path.join(d, f)
            for m in USE.finditer(open(p, errors="replace").read()):
                found.setdefault(m.group(1), os.path.relpath(p, root))
    return found


def documented(root):
    doc = set()
    for prog in ("bcpd", "bcp-cli", "bcp-tx", "bcp-seeder", "bench_bcp"):
        exe = os.path.join(root, "bin", prog)
        if not os.path.exists(exe):
            continue
        r = subprocess.run([exe, "-help", "-help-debug"], capture_output=True, text=True, timeout=60)
        text = r.stdout + r.stderr
        for m in HELP.finditer(text):
            doc.add(m.group(1).split("=")[0].split("<")[0])
        for line in text.splitlines():
            if "Usage:" in line or line.startswith(" " * 8):
                for m in USAGE.finditer(line):
                    doc.add(m.group(1).split("=")[0])
    return doc


def reference_options(root):
    out = {}
    for line in open(os.path.join(root, "contrib", "devtools", "reference_options.txt")):
        if line.strip() and not line.startswith("#"):
            name, where = line.split()
            out[name] = where
    return out


def main(argv):
    check_ref = "--reference" in argv
    argv = [a for a in argv if a != "--reference"]
    root = argv[0] if argv else os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    used = used_options(root)
    doc = documented(root)
    missing = sorted(o for o in used if o not in doc and o not in UNDOCUMENTED)
    for o in missing:
        print(f"undocumented option {o} (read in {used[o]})")
    print(f"{len(used)} options read, {len(doc)} documented, {len(missing)} undocumented")
    bad = len(missing)
    if check_ref:
        ref = reference_options(root)
        absent = sorted(o for o in ref if o not in used and o not in doc and o not in REFERENCE_NOT_APPLICABLE)
        for o in absent:
            print(f"reference option {o} (read in {ref[o]}) is neither read nor documented here")
        print(f"{len(ref)} reference options, {len(absent)} missing")
        bad += len(absent)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
