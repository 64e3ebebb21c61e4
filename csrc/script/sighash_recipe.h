// Host side of the device FORKID signature hash (K7, kernels/sighash_device.h): turns a
// (transaction, input, script code, hash type, amount) check into the recipe the GPU hashes.
// Parity: reference src/script/interpreter.cpp:1354-1404 (SignatureHash, SIGHASH_FORKID branch);
// the hash-type rules (which of hashPrevouts / hashSequence / hashOutputs are blanked) are
// resolved here, so the device only concatenates and hashes.
#pragma once
#include "kernels/gpu_api.h"
#include "primitives/transaction.h"
#include "script/interpreter.h"

namespace bcp {

// Shared per-transaction fields (version, the three BIP143 hashes, lock time).
void FillSighashTx(const CTransaction& tx, const PrecomputedTransactionData& txdata, gpu::SighashTx& out);

// One check. Returns false when the digest is not a FORKID digest the recipe can express
// (legacy digests, out-of-range inputs, SIGHASH_SINGLE with a matching output): the caller then
// computes SignatureHash on the CPU and marks the job SIGHASH_JOB_PRECOMPUTED.
bool FillSighashJob(const CTransaction& tx, unsigned int nIn, uint32_t nHashType, Amount amount, uint32_t flags,
                    uint32_t txIndex, uint32_t codeOff, uint32_t codeLen, gpu::SighashJob& job);

// CPU evaluation of a recipe (tests and the device-fault fallback): the same bytes the kernel
// hashes.
uint256 SighashFromRecipe(const gpu::SighashTx& tx, const gpu::SighashJob& job, const unsigned char* code);

} // namespace bcp
