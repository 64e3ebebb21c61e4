#!/usr/bin/env python3
"""List the block hashes of the best chain, in height order, over JSON-RPC
(reference contrib/linearize/linearize-hashes.py).

    linearize-hashes.py CONFIG-FILE > hashlist.txt

CONFIG-FILE holds key=value lines: host (127.0.0.1), port (8332-style RPC port), rpcuser,
rpcpassword, min_height (0), max_height (tip), rev_hash_bytes (false).
"""
import base64
import http.client
import json
import sys


def read_config(path):
    settings = {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            k, v = line.split("=", 1)
            settings[k.strip()] = v.strip()
    return settings


class RPC:
    def __init__(self, host, port, user, password):
        self.host, self.port = host, int(port)
        self.auth = "Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()

    def batch(self, calls):
        body = json.dumps([{"version": "1.1", "method": m, "params": p, "id": i} for i, (m, p) in enumerate(calls)])
        c = http.client.HTTPConnection(self.host, self.port, timeout=60)
        c.request("POST", "/", body, {"Authorization": self.auth, "Content-Type": "application/json"})
        r = json.loads(c.getresponse().read())
        c.close()
        return [x["result"] for x in sorted(r, key=lambda x: x["id"])]


def get_hashes(settings, out=sys.stdout):
    rpc = RPC(settings.get("host", "127.0.0.1"), settings["port"], settings["rpcuser"], settings["rpcpassword"])
    lo = int(settings.get("min_height", 0))
    hi = int(settings["max_height"]) if "max_height" in settings else rpc.batch([("getblockcount", [])])[0]
    rev = settings.get("rev_hash_bytes", "false").lower() == "true"
    hashes = []
    for start in range(lo, hi + 1, 1000):
        for h in rpc.batch([("getblockhash", [n]) for n in range(start, min(start + 1000, hi + 1))]):
            if rev:
                h = bytes.fromhex(h)[::-1].hex()
            hashes.append(h)
            out.write(h + "\n")
    return hashes


if __name__ == "__main__":
    if len(sys.argv) != 2:
        print(__doc__, file=sys.stderr)
        sys.exit(1)
    get_hashes(read_config(sys.argv[1]))
