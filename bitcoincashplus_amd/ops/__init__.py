"""Python front-ends for the gfx950 kernels (csrc/kernels/*.hip).

Each op runs on the MI355X and raises if no HIP device is visible — there is no
silent CPU fallback.  Ops that have a CPU implementation in the native core take
an explicit ``use_gpu=False``.  Tensor inputs (``torch.uint8``) are accepted
where batches are naturally dense.  They are flattened to host bytes here
(``.cpu()`` — a pageable copy); the native layer then packs them into per-device
pinned staging buffers that it keeps across calls (``HostBuf`` in
csrc/kernels/hip_util.h), so each H2D/D2H transfer is a single DMA from pinned
memory on the op's own non-blocking stream.

Kernel map (reference hot loops):
  sha256d64          K6  SHA-256d of 64-byte nodes (merkle levels)  sha256.hip
  sha256d_batch      K6  txid-style SHA-256d of variable messages   sha256.hip
  merkle_root        K6  whole-tree reduction on device              sha256.hip
  scan_nonces        K5  legacy SHA-256d header nonce scan           sha256.hip
  equihash_verify    K4  batched IsValidSolution                     equihash_verify.hip
  ecdsa_verify       K8  batched secp256k1 verify                    secp256k1.hip
  verify_forkid      K8  block-path deferred checks -> verify batch  secp256k1.hip (GpuVerifyDeferred)
  short_txids        K9  BIP152 SipHash-2-4 short ids                relay.hip
  Equihash solving (K1-K3) is ``models.EquihashModel.gpu_solver``.
"""
from __future__ import annotations

from typing import Iterable, Sequence

from .._native import native, require_gpu

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def _as_bytes(x) -> bytes:
    if torch is not None and isinstance(x, torch.Tensor):
        if x.dtype != torch.uint8:
            raise TypeError("expected a torch.uint8 tensor")
        return x.detach().contiguous().cpu().numpy().tobytes()
    return bytes(x)


def sha256d64(data, device: int = -1):
    """SHA-256d of consecutive 64-byte blocks. Returns bytes, or a [N,32] uint8 tensor
    when given a tensor."""
    require_gpu("sha256d64")
    raw = _as_bytes(data)
    if len(raw) % 64:
        raise ValueError("input length must be a multiple of 64")
    out = native.sha256d64_batch_gpu(raw, device)
    if torch is not None and isinstance(data, torch.Tensor):
        return torch.frombuffer(bytearray(out), dtype=torch.uint8).view(-1, 32).to(data.device)
    return out


def sha256d_batch(msgs: Sequence[bytes], device: int = -1) -> list:
    require_gpu("sha256d_batch")
    return native.sha256d_batch_gpu([bytes(m) for m in msgs], device)


def merkle_root(leaves, device: int = -1):
    """Merkle root of 32-byte leaves on device. Returns (root, mutated) like the
    reference ComputeMerkleRoot (consensus/merkle.cpp)."""
    require_gpu("merkle_root")
    raw = _as_bytes(leaves) if not isinstance(leaves, (list, tuple)) else b"".join(leaves)
    if len(raw) % 32:
        raise ValueError("leaves must be 32-byte hashes")
    return native.merkle_root_gpu(raw, device)


def scan_nonces(header80: bytes, target_le: bytes, start: int, count: int, device: int = -1) -> int:
    """First nonce in [start, start+count) whose legacy header hash <= target, or -1."""
    require_gpu("scan_nonces")
    return native.sha256d_scan_nonces_gpu(bytes(header80), bytes(target_le), start, count, device)


def equihash_verify(n: int, k: int, states, solutions, device: int = -1) -> list:
    require_gpu("equihash_verify")
    return native.eh_verify_batch_gpu(n, k, list(states), [bytes(s) for s in solutions], device)


def ecdsa_verify(items: Iterable, use_gpu: bool = True, threads: int = 8):
    """Batched ECDSA verify of (pubkey, der_sig, sighash32) triples.
    Returns (list[bool], milliseconds)."""
    if use_gpu:
        require_gpu("ecdsa_verify")
    return native.ecdsa_verify_batch([(bytes(a), bytes(b), bytes(c)) for a, b, c in items], use_gpu, threads)


__all__ = ["sha256d64", "sha256d_batch", "merkle_root", "scan_nonces", "equihash_verify", "ecdsa_verify"]


def short_txids(k0: int, k1: int, txids, device: int = -1) -> list:
    """48-bit BIP152 short ids of 32-byte txids (bytes of N*32, a list of 32-byte hashes, or a
    [N,32] uint8 tensor) under the SipHash key (k0, k1)."""
    require_gpu("short_txids")
    if isinstance(txids, (list, tuple)):
        txids = b"".join(txids)
    raw = _as_bytes(txids)
    if len(raw) % 32:
        raise ValueError("txids must be 32-byte hashes")
    return native.short_txid_batch_gpu(k0, k1, raw, device)


def verify_forkid(items: Iterable, use_gpu: bool = True):
    """Block-path signature checks (pubkey, sig_with_hashtype, script_code, tx_bytes, n_in,
    amount) through the node's deferring checker (the digest computed as a script worker does)
    and the GPU verify batch. Returns (results, digests)."""
    if use_gpu:
        require_gpu("verify_forkid")
    return native.verify_sig_deferred(list(items), use_gpu=use_gpu)
