"""Python front-ends for the gfx950 kernels (csrc/kernels/*.hip).

Each op runs on the MI355X and raises if no HIP device is visible — there is no
silent CPU fallback.  Ops that have a CPU implementation in the native core take
an explicit ``use_gpu=False``.

Two input paths:
* **Device-resident** (``torch.uint8`` tensors on the GPU): ``sha256d64``,
  ``short_txids`` and ``ecdsa_verify_compact`` hand the tensors' device pointers to
  the kernels and enqueue them on the tensors' current torch stream
  (``torch.cuda.current_stream().cuda_stream``).  Results come back as GPU tensors;
  nothing is copied to the host and nothing synchronises, so the ops compose with
  other GPU work on the same stream (``gpu_api.h`` "device-resident entry points").
* **Host** (bytes, lists, CPU tensors): packed into per-device pinned staging
  buffers kept across calls (``HostBuf`` in csrc/kernels/hip_util.h), one H2D and one
  D2H DMA per call on the op's own non-blocking stream.

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


def _on_gpu(x) -> bool:
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def _u8(x, what: str):
    if x.dtype != torch.uint8:
        raise TypeError(f"{what}: expected a torch.uint8 tensor")
    return x.detach().contiguous()


def _dev_stream(t):
    """(device index, stream handle) of the current torch stream on t's device."""
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    return dev, torch.cuda.current_stream(dev).cuda_stream


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
    if _on_gpu(data):
        x = _u8(data, "sha256d64").view(-1)
        if x.numel() % 64:
            raise ValueError("input length must be a multiple of 64")
        n = x.numel() // 64
        out = torch.empty((n, 32), dtype=torch.uint8, device=x.device)
        dev, stream = _dev_stream(x)
        native.sha256d64_device(x.data_ptr(), out.data_ptr(), n, dev, stream)
        return out
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


__all__ = ["sha256d64", "sha256d_batch", "merkle_root", "scan_nonces", "equihash_verify", "ecdsa_verify",
           "ecdsa_verify_compact", "short_txids", "verify_forkid"]


def short_txids(k0: int, k1: int, txids, device: int = -1) -> list:
    """48-bit BIP152 short ids of 32-byte txids (bytes of N*32, a list of 32-byte hashes, or a
    [N,32] uint8 tensor) under the SipHash key (k0, k1)."""
    require_gpu("short_txids")
    if _on_gpu(txids):
        x = _u8(txids, "short_txids").view(-1)
        if x.numel() % 32:
            raise ValueError("txids must be 32-byte hashes")
        if x.data_ptr() % 16:
            x = x.clone()  # the kernel reads 16-byte words
        n = x.numel() // 32
        out = torch.empty(n, dtype=torch.int64, device=x.device)  # 48-bit ids
        dev, stream = _dev_stream(x)
        native.short_txids_device(k0, k1, x.data_ptr(), out.data_ptr(), n, dev, stream)
        return out
    if isinstance(txids, (list, tuple)):
        txids = b"".join(txids)
    raw = _as_bytes(txids)
    if len(raw) % 32:
        raise ValueError("txids must be 32-byte hashes")
    return native.short_txid_batch_gpu(k0, k1, raw, device)


def ecdsa_verify_compact(msg32, sig64, pub33):
    """Batched verify of packed signatures: msg32 [N,32] digests, sig64 [N,64] compact r||s
    (low S: a high-S signature is reported invalid, as secp256k1_ecdsa_verify does), pub33
    [N,33] compressed keys. GPU tensors stay on the device and give a [N] uint8
    GPU tensor (1 = valid) on the current stream; bytes give a list of bools through the
    node's verify lanes."""
    require_gpu("ecdsa_verify_compact")
    if _on_gpu(msg32):
        m, s_, p = _u8(msg32, "msg32").view(-1), _u8(sig64, "sig64").view(-1), _u8(pub33, "pub33").view(-1)
        n = m.numel() // 32
        if m.numel() != n * 32 or s_.numel() != n * 64 or p.numel() != n * 33:
            raise ValueError("msg32/sig64/pub33 sizes")
        if not (s_.device == m.device == p.device):
            raise ValueError("inputs on different devices")
        out = torch.empty(n, dtype=torch.uint8, device=m.device)
        jobs = torch.empty(max(n, 1) * native.ecdsa_job_bytes(), dtype=torch.uint8, device=m.device)
        dev, stream = _dev_stream(m)
        native.ecdsa_verify_device(m.data_ptr(), s_.data_ptr(), p.data_ptr(), jobs.data_ptr(), out.data_ptr(), n,
                                   dev, stream)
        return out
    return native.gpu_verify_ecdsa_packed(_as_bytes(msg32), _as_bytes(sig64), _as_bytes(pub33))


def verify_forkid(items: Iterable, use_gpu: bool = True):
    """Block-path signature checks (pubkey, sig_with_hashtype, script_code, tx_bytes, n_in,
    amount) through the node's deferring checker (the digest computed as a script worker does)
    and the GPU verify batch. Returns (results, digests)."""
    if use_gpu:
        require_gpu("verify_forkid")
    return native.verify_sig_deferred(list(items), use_gpu=use_gpu)
