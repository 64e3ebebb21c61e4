// Host-side API of the CDNA4 (gfx950) kernels. Every function here is
// implemented in a csrc/kernels/*.hip translation unit and launches hand-written
// HIP kernels; nothing here falls back to the CPU. Callers that must run
// without a GPU (the node on a CPU-only host) check GpuAvailable() first and
// use the CPU consensus code instead.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <functional>
#include <vector>

namespace bcp {
class CBlake2b;
namespace gpu {

bool GpuAvailable();
int DeviceCount();
std::string DeviceName(int device);
// Throws std::runtime_error with the HIP error string.
void Check(int hip_status, const char* what);

// --------------------------------------------------------------- Equihash
// Host mirror of bcpk::EhBaseState (csrc/kernels/blake2b_device.h).
struct EhBaseState {
    uint64_t h[8];
    uint64_t m[16];
    uint64_t t0;
    uint32_t g_byte;
    uint32_t outlen;
};
// Build the g-independent state from a BLAKE2b state that already absorbed
// CEquihashInput || nNonce (the solver/verifier then appends le32(g)).
EhBaseState MakeEhBaseState(const CBlake2b& st);
// Bytes of a minimal-encoded (N, K) solution (1344 for (200, 9)).
size_t EquihashSolutionBytes(unsigned N, unsigned K);

struct EhGpuStats {
    uint64_t nonces = 0;
    uint64_t candidates = 0;
    uint64_t duplicates = 0;
    uint64_t solutions = 0;
    uint64_t dropped_rows = 0;   // rows lost to bucket overflow (debug mode, nonce 0 of each batch)
    uint64_t cand_dropped = 0;   // final-round candidates past the per-nonce list (MAXCAND), every nonce
    uint64_t cand_max = 0;       // largest per-nonce final-round candidate count seen
    double gpu_ms = 0;
    std::vector<uint64_t> stage_rows, stage_dropped, stage_maxfill; // debug mode, last batch
    std::vector<std::vector<uint64_t>> stage_top;
    std::vector<uint64_t> pair_dropped;
    std::vector<uint64_t> stage_dropped_all;  // every nonce: rows past a round's capacity per stage (accumulated)
    std::vector<uint64_t> pair_dropped_all;   // every nonce: pairs past a round's pair list, per round (accumulated)
    std::vector<uint64_t> stage_maxfill_all;  // debug: fullest bucket per stage, last batch
    std::vector<uint64_t> overflow_fills; // debug: (stage << 32 | fill) of every bucket past its capacity (accumulated)
    std::vector<std::vector<uint32_t>> debug_cands;                  // debug: every candidate of nonce 0 (valid or not)
};

// Batched Equihash solver: one launch sequence solves `batch` nonces at once
// (8 + 3 kernels per batch, bucket-per-workgroup collision rounds in LDS).
class EquihashGpuSolver {
public:
    EquihashGpuSolver(unsigned n, unsigned k, int batch, int device = -1);
    ~EquihashGpuSolver();
    unsigned N() const;
    unsigned K() const;
    int Batch() const;
    // states.size() <= batch. Returns, per nonce, canonical index lists of all
    // valid (distinct-index) solutions found.
    std::vector<std::vector<std::vector<uint32_t>>> Solve(const std::vector<EhBaseState>& states);
    // Asynchronous split used by the pipelined miner/bench: Launch enqueues the
    // whole sequence on the solver's stream; Collect waits and decodes.
    void Launch(const std::vector<EhBaseState>& states);
    // The same, pipelined behind `prev` (another solver on the same device whose batch was
    // launched just before this one): this batch's generation starts once prev's generation is
    // done, and its collision rounds once prev's rounds are done. Generation (VALU-bound) then
    // runs beside the previous batch's rounds (LDS/latency-bound) instead of beside another
    // generation.
    void Launch(const std::vector<EhBaseState>& states, const EquihashGpuSolver& prev);
    std::vector<std::vector<std::vector<uint32_t>>> Collect();
    const EhGpuStats& Stats() const;
    void SetDebug(bool on);   // collect per-stage bucket statistics (extra D2H copies)
    void SetStampMode(bool on); // diagnostic: launch phase-timestamped round kernels
    std::vector<uint64_t> DebugDump(); // diagnostic: leaf indices + parent triples of nonce 0
    // Test hook (after a Solve): re-run the tree expansion of nonce 0's candidates with the first
    // candidate's left stage-(K-1) parent corrupted - mode 1: bucket out of range, mode 2: LDS
    // row out of range, 0: untouched. Returns each candidate's valid flag; the expansion must
    // reject the corrupted candidate without touching memory outside the stage arrays.
    std::vector<uint32_t> DebugExpandCorrupt(int mode);
    std::vector<std::vector<double>> PhaseCycles(int nonces);
    void ResetStats();
    size_t DeviceBytes() const;
    struct Impl;
private:
    std::unique_ptr<Impl> impl;
};

// Batched consensus verifier (reference CheckEquihashSolution / IsValidSolution).
// One workgroup per solution: 2^K lanes hash their index, LDS tree reduction.
std::vector<uint8_t> EquihashVerifyBatch(unsigned n, unsigned k, const std::vector<EhBaseState>& states,
                                         const std::vector<std::vector<unsigned char>>& solutions,
                                         int device = -1);

// --------------------------------------------------------------- SHA-256d
// out[i] = SHA256d(in[offs[i] .. offs[i]+lens[i]))
std::vector<unsigned char> Sha256dBatch(const std::vector<unsigned char>& data, const std::vector<uint64_t>& offs,
                                        const std::vector<uint32_t>& lens, int device = -1);
// out[i] = SHA256d(in[64*i .. 64*i+64))
std::vector<unsigned char> Sha256d64Batch(const std::vector<unsigned char>& data, int device = -1);
// Merkle root of 32-byte leaves with the reference's mutation flag
// (reference src/consensus/merkle.cpp:47-175, CVE-2012-2459).
std::vector<unsigned char> MerkleRoot(const std::vector<unsigned char>& leaves, bool* mutated, int device = -1);
// Legacy 80-byte header nonce sweep: returns the first nonce in
// [start, start+count) with SHA256d(header) <= target, or -1.
int64_t Sha256dScanNonces(const unsigned char header80[80], const unsigned char target_le[32], uint32_t start,
                          uint64_t count, int device = -1);

// --------------------------------------------------------------- relay: BIP152 short ids
// out[i] = SipHash-2-4(k0, k1, txid_i) & (2^48 - 1), txids32 = n x 32 bytes (reference
// src/blockencodings.cpp:37-42 GetShortID, src/hash.cpp:181-300 SipHashUint256). Used for the
// mempool side of compact-block reconstruction when the pool is large.
std::vector<uint64_t> ShortTxIdBatch(uint64_t k0, uint64_t k1, const unsigned char* txids32, size_t n,
                                     int device = -1);

// --------------------------------------------------------------- secp256k1
// ECDSA verification batch: N jobs, msg32 = N*32 (big-endian digest bytes as signed),
// sig64 = N*64 (r||s big-endian, s low-S-normalised, r,s in [1,n-1] checked on host),
// pub33 = N*33 compressed keys (0x02/0x03 || x; the host converts uncompressed/hybrid
// keys after its on-curve check). The GPU decompresses, computes u1*G + u2*Q and
// compares x(R) mod n with r. result[i] = 1 iff valid. Batches below the GPU
// threshold should stay on the CPU (launch latency ~10 us).
std::vector<uint8_t> EcdsaVerifyBatch(const std::vector<unsigned char>& msg32, const std::vector<unsigned char>& sig64,
                                      const std::vector<unsigned char>& pub33, int device = -1);

// Batches of at most EcdsaFusedMax() signatures run one fused latency kernel (scalar work,
// key decompression and the two GLV halves on separate waves, 10 x 26-bit field); larger ones
// the prep + verify throughput kernels. Process-wide; the default is measured
// (profiles/ecdsa_r5.md).
void SetEcdsaFusedMax(size_t n);
size_t EcdsaFusedMax();
// Verify kernel of the split (prep + verify) path: 0 = 8 x 32-bit field with an inverted
// table, 1 = 10 x 26-bit field with the global-z table (one lane per signature for whole rounds
// of the device, one GLV half per lane for a last round at most half full), 2 / 3 = only the
// one-lane / only the half-lane 10 x 26 kernel (tests pin each).
void SetEcdsaSplitKernel(int k);
int EcdsaSplitKernel();

// --------------------------------------------------------------- device-resident entry points
// The tensor API (bitcoincashplus_amd.ops with torch tensors on the GPU): every pointer is
// device memory on `device`, the kernels are enqueued on `stream` (a hipStream_t passed as an
// integer, e.g. torch.cuda.current_stream().cuda_stream) after the work already queued there,
// and nothing is copied or synchronised. The caller keeps the buffers alive until the stream
// has run (torch's caching allocator does this for tensors used on their own stream).
// out32[i] = SHA256d(in64[64*i .. 64*i+64))
void Sha256d64Device(const void* in64, void* out32, size_t n, int device, uintptr_t stream);
// out[i] = BIP152 short id of txid i (48 bits in a uint64); txids32 16-byte aligned
void ShortTxIdsDevice(uint64_t k0, uint64_t k1, const void* txids32, void* out64, size_t n, int device,
                      uintptr_t stream);
// Device scratch the ECDSA kernels need per signature (the prep kernel's job records).
size_t EcdsaJobBytes();
// result[i] = 1 iff signature i verifies; inputs as EcdsaVerifyBatch (msg32 n x 32, sig64 compact
// r||s n x 64, pub33 compressed n x 33), jobs = n x EcdsaJobBytes() of scratch.
void EcdsaVerifyDevice(const void* msg32, const void* sig64, const void* pub33, void* jobs, void* result, size_t n,
                       int device, uintptr_t stream);

// --------------------------------------------------------------- verification lanes
// A verification lane is one device plus one HIP stream (created at the device's greatest
// priority when `highPriority`, so a validation batch is scheduled ahead of the persistent
// solver kernels the miner keeps on the same device) plus grow-only pinned host staging and
// device buffers that every batch reuses (one H2D and one D2H copy per batch, no pageable
// transfers, no per-batch allocation). A lane is driven by one thread at a time; the node's
// GpuVerifyService gives each lane its own service thread (csrc/node/gpuverify.h).
class VerifyLane {
public:
    VerifyLane(int device, bool highPriority);
    ~VerifyLane();
    VerifyLane(const VerifyLane&) = delete;
    VerifyLane& operator=(const VerifyLane&) = delete;
    int Device() const;
    int Priority() const;
    // Same contract as EcdsaVerifyBatch: n packed jobs, result[i] = 1 iff valid.
    void Ecdsa(const unsigned char* msg32, const unsigned char* sig64, const unsigned char* pub33, size_t n,
               uint8_t* result);
    // Same, with the inputs written by `fill` straight into the lane's pinned staging buffer
    // (msg32: n x 32 B, sig64: n x 64 B, pub33: n x 33 B) instead of being copied there.
    void EcdsaFill(size_t n, const std::function<void(unsigned char* msg32, unsigned char* sig64,
                                                        unsigned char* pub33)>& fill,
                   uint8_t* result);
    // Same with DER signatures parsed on the device: sig73 holds n slots of [length byte][up to
    // 72 DER bytes] (hash type stripped), parsed with the reference's lax rules
    // (src/pubkey.cpp ecdsa_signature_parse_der_lax) and low-S normalised by the prep kernel; a
    // signature that does not parse verifies false. (The host then only copies bytes.)
    static constexpr size_t DER_SLOT = 73;
    void EcdsaDerFill(size_t n, const std::function<void(unsigned char* msg32, unsigned char* sig73,
                                                           unsigned char* pub33)>& fill,
                      uint8_t* result);
    // n block headers: fill(in140, sols, lenok) writes each header's 140-byte Equihash input
    // (CEquihashInput || nNonce), its solution (EquihashSolutionBytes bytes) and whether the
    // solution had that length into the lane's pinned staging; the device builds the BLAKE2b
    // base states and verifies. result[i] = 1 iff header i's solution is valid.
    void EquihashHeaders(unsigned N, unsigned K, size_t n,
                         const std::function<void(uint8_t* in140, uint8_t* sols, uint8_t* lenok)>& fill,
                         uint8_t* result);
    // Same contract as EquihashVerifyBatch for n (state, solution) pairs; a solution of the
    // wrong length is rejected.
    void Equihash(unsigned N, unsigned K, const EhBaseState* states, const std::vector<unsigned char>* const* sols,
                  size_t n, uint8_t* result);
    // Batches and items this lane has run (service statistics).
    uint64_t Batches() const;
    uint64_t Items() const;
    // time spent in the callers' fills (host) and in copies + kernels + the wait (device)
    uint64_t FillMicros() const;
    uint64_t DeviceMicros() const;
    struct Impl;

private:
    std::unique_ptr<Impl> impl;
};

} // namespace gpu
} // namespace bcp
