#!/usr/bin/env python3
"""Pick fixed seed candidates from a DNS seeder dump.

    contrib/seeds/makeseeds.py < dnsseed.dump > contrib/seeds/nodes_main.txt

Reads the `-dumpfile` written by bcp-seeder (csrc/tools/bcp-seeder.cpp). Its columns are:
address, good, lastSuccess, %(2h) uptime, blocks, service bits (hex), protocol version, and the
quoted user agent. A node is kept only if all of these hold:

* the seeder marks it good;
* its 2-hour uptime is at least 50 %;
* it reports the NODE_NETWORK service bit;
* its height is at least --min-blocks;
* its protocol version is at least 70016 (the BCP header format);
* its user agent matches --agent.

At most --per-net16 nodes are kept per IPv4 /16 (or IPv6 /32), so one hoster cannot fill the
list. The best --max nodes by uptime, then height, are printed in the nodes_*.txt format.

Parity: reference contrib/seeds/makeseeds.py (same filters: uptime, service bits, minimum
height, user-agent pattern, per-network diversity. It limits per ASN; this tool has no network
access for ASN lookups, so it limits per address prefix).
"""
import argparse
import ipaddress
import re
import sys

NODE_NETWORK = 1
MIN_PROTOCOL = 70016


def parse_line(line):
    line = line.strip()
    if not line or line.startswith("#"):
        return None
    m = re.match(r'^(\S+)\s+(\d+)\s+(\d+)\s+([\d.]+)%\s+(\d+)\s+([0-9a-fA-F]+)\s+(\d+)\s+"(.*)"$', line)
    if not m:
        return None
    addr, good, last, uptime, blocks, svcs, version, agent = m.groups()
    host, _, port = addr.rpartition(":")
    host = host.strip("[]")
    try:
        ip = ipaddress.ip_address(host)
    except ValueError:
        ip = None  # onion or unparsable: kept only by address, no prefix limit
    return {"addr": addr, "ip": ip, "port": int(port) if port.isdigit() else 0, "good": good == "1",
            "last": int(last), "uptime": float(uptime), "blocks": int(blocks), "services": int(svcs, 16),
            "version": int(version), "agent": agent}


def net_key(n):
    ip = n["ip"]
    if ip is None:
        return n["addr"]
    if ip.version == 4:
        return str(ipaddress.ip_network(f"{ip}/16", strict=False))
    return str(ipaddress.ip_network(f"{ip}/32", strict=False))


def select(nodes, min_blocks, agent, per_net, max_nodes):
    pat = re.compile(agent)
    ok = [n for n in nodes if n and n["good"] and n["uptime"] >= 50.0 and n["services"] & NODE_NETWORK and
          n["blocks"] >= min_blocks and n["version"] >= MIN_PROTOCOL and pat.search(n["agent"])]
    ok.sort(key=lambda n: (-n["uptime"], -n["blocks"], n["addr"]))
    per = {}
    out = []
    for n in ok:
        k = net_key(n)
        if per.get(k, 0) >= per_net:
            continue
        per[k] = per.get(k, 0) + 1
        out.append(n)
        if len(out) >= max_nodes:
            break
    return out


def main(argv):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--min-blocks", type=int, default=0)
    ap.add_argument("--agent", default=r"Bitcoin Cash Plus|BCP|bcp")
    ap.add_argument("--per-net16", type=int, default=2)
    ap.add_argument("--max", type=int, default=512)
    a = ap.parse_args(argv)
    nodes = [parse_line(l) for l in sys.stdin]
    for n in select(nodes, a.min_blocks, a.agent, a.per_net16, a.max):
        print(n["addr"])
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
