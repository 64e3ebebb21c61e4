"""Network "model families": the chain parameter sets and the proof-of-work models.

A BCP deployment is selected by two things — the chain (main / test / regtest,
reference src/chainparams.cpp) and the PoW it runs: SHA-256d before ``BCPHeight``
and Equihash(n, k) after it (reference src/crypto/equihash.h:197-200 instantiates
(96,3), (200,9), (96,5), (48,5)).  ``ChainModel`` reads the parameters from the
native core (one source of truth with bcpd); ``EquihashModel`` describes a
parameter set and builds its CPU/GPU solver and verifier.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from .._native import native, require_gpu

GPU_EQUIHASH = {(200, 9), (96, 5), (48, 5)}
CPU_EQUIHASH = {(200, 9), (96, 5), (96, 3), (48, 5)}


@dataclass(frozen=True)
class EquihashModel:
    n: int
    k: int

    def __post_init__(self):
        if (self.n, self.k) not in CPU_EQUIHASH:
            raise ValueError(f"unsupported Equihash parameters ({self.n},{self.k})")

    @property
    def collision_bits(self) -> int:
        return self.n // (self.k + 1)

    @property
    def indices_per_solution(self) -> int:
        return 1 << self.k

    @property
    def solution_bytes(self) -> int:
        # minimal encoding: 2^k indices of (collision_bits + 1) bits
        return self.indices_per_solution * (self.collision_bits + 1) // 8

    @property
    def initial_rows(self) -> int:
        return 1 << (self.collision_bits + 1)

    @property
    def gpu_supported(self) -> bool:
        return (self.n, self.k) in GPU_EQUIHASH

    def state(self, data: bytes = b"") -> "native.EquihashState":
        st = native.EquihashState(self.n, self.k)
        if data:
            st.update(data)
        return st

    def solve_cpu(self, state):
        """Reference-equivalent CPU solve (reference equihash.cpp:332 BasicSolve)."""
        sols, _ = native.eh_solve_cpu(self.n, self.k, state)
        return sols

    def verify(self, state, solution: bytes) -> bool:
        ok, _ = native.eh_is_valid_solution(self.n, self.k, state, solution)
        return bool(ok)

    def gpu_solver(self, batch: int = 8, device: int = 0):
        if not self.gpu_supported:
            raise ValueError(f"no GPU solver for ({self.n},{self.k})")
        require_gpu(f"Equihash({self.n},{self.k}) GPU solver")
        return native.EquihashGpuSolver(self.n, self.k, batch, device)

    def verify_batch_gpu(self, states, solutions, device: int = 0):
        require_gpu("Equihash GPU verifier")
        return native.eh_verify_batch_gpu(self.n, self.k, list(states), list(solutions), device)


@dataclass(frozen=True)
class ChainModel:
    network: str
    params: dict = field(repr=False, compare=False)

    @classmethod
    def load(cls, network: str) -> "ChainModel":
        return cls(network, dict(native.chain_params(network)))

    @property
    def equihash(self) -> EquihashModel:
        return EquihashModel(self.params["equihash_n"], self.params["equihash_k"])

    @property
    def bcp_height(self) -> int:
        return self.params["bcp_height"]

    def pow_for_height(self, height: int) -> str:
        """'sha256d' for legacy blocks, 'equihash' from BCPHeight on."""
        return "equihash" if height >= self.bcp_height else "sha256d"

    def header_size(self, height: int) -> int:
        return 140 if height >= self.bcp_height else 80

    def __getitem__(self, key):
        return self.params[key]


MODELS = {
    "equihash_200_9": EquihashModel(200, 9),
    "equihash_96_5": EquihashModel(96, 5),
    "equihash_96_3": EquihashModel(96, 3),
    "equihash_48_5": EquihashModel(48, 5),
}


def chain(network: str) -> ChainModel:
    return ChainModel.load(network)


__all__ = ["EquihashModel", "ChainModel", "MODELS", "chain", "GPU_EQUIHASH"]
