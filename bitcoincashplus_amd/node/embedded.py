"""In-process node: the C++ chainstate/mempool/RPC table driven from Python.

Every RPC registered in csrc/rpc/*.cpp is reachable as a method:
    node = EmbeddedNode("regtest", datadir)
    node.generate(10); node.getblockcount()
Errors are raised as RPCError(code, message), mirroring the JSON-RPC server.
"""
from __future__ import annotations

import json

from .._native import native


class RPCError(Exception):
    def __init__(self, code, message):
        super().__init__(f"{code}: {message}")
        self.code = code
        self.message = message


class EmbeddedNode:
    def __init__(self, chain="regtest", datadir=".", memory=False, gpu=False, args=()):
        native.node_start(chain, datadir, memory, gpu, list(args))
        self.chain = chain
        self.datadir = datadir

    def call(self, method, *params):
        reply = json.loads(native.rpc_json(method, json.dumps(list(params))))
        if reply.get("error"):
            raise RPCError(reply["error"]["code"], reply["error"]["message"])
        return reply["result"]

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return lambda *p: self.call(name, *p)

    def stop(self):
        native.node_stop()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()
