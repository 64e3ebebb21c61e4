"""bitcoincashplus_amd — an MI355X-native Bitcoin Cash Plus node, miner and verifier.

Layout (mirrors the reference's capabilities, not its code):

* ``_bcpnative`` (C++/HIP extension, built from ``csrc/``): consensus core, Equihash,
  script interpreter, secp256k1, chainstate/mempool/miner, RPC/P2P node, and the
  gfx950 kernels (Equihash solve/verify, SHA-256d, ECDSA).
* ``models/``   network "model families": chain parameters (main/test/regtest) and the
  Equihash parameter sets, each with its solver/verifier configuration.
* ``ops/``      Python front-ends for the HIP kernels (torch-stream aware).
* ``parallel/`` one-process-per-GPU scale-out over ``torch.distributed`` (RCCL over xGMI):
  nonce-space data parallel mining and sharded batch verification.
* ``node/``     process management for the native ``bcpd`` daemon and an RPC client.
* ``utils/``    serialization helpers, a pure-Python P2P test peer, test framework.
"""
from ._native import native, gpu_available, require_gpu  # noqa: F401

__version__ = "0.17.0-mi355x.1"
