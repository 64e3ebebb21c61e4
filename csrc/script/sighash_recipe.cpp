#include "script/sighash_recipe.h"

#include "crypto/hashes.h"
#include "primitives/serialize.h"

#include <cstring>

namespace bcp {

namespace {
void PutLE32(unsigned char* p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (unsigned char)(v >> (8 * i));
}
} // namespace

void FillSighashTx(const CTransaction& tx, const PrecomputedTransactionData& txdata, gpu::SighashTx& out) {
    PutLE32(out.version, (uint32_t)tx.nVersion);
    memcpy(out.hashPrevouts, txdata.hashPrevouts.begin(), 32);
    memcpy(out.hashSequence, txdata.hashSequence.begin(), 32);
    memcpy(out.hashOutputs, txdata.hashOutputs.begin(), 32);
    PutLE32(out.lockTime, tx.nLockTime);
}

bool FillSighashJob(const CTransaction& tx, unsigned int nIn, uint32_t nHashType, Amount amount, uint32_t flags,
                    uint32_t txIndex, uint32_t codeOff, uint32_t codeLen, gpu::SighashJob& job) {
    if (!(nHashType & SIGHASH_FORKID) || !(flags & SCRIPT_ENABLE_SIGHASH_FORKID)) return false; // legacy digest
    if (nIn >= tx.vin.size()) return false;
    const uint32_t base = nHashType & 0x1f;
    // SIGHASH_SINGLE with a matching output hashes that one output: the CPU supplies the digest
    if (base == SIGHASH_SINGLE && nIn < tx.vout.size()) return false;
    memset(&job, 0, sizeof(job));
    job.tx = txIndex;
    job.codeOff = codeOff;
    job.codeLen = codeLen;
    job.hashType = nHashType;
    if (nHashType & SIGHASH_ANYONECANPAY) job.flags |= gpu::SIGHASH_JOB_ZERO_PREVOUTS | gpu::SIGHASH_JOB_ZERO_SEQUENCE;
    if (base == SIGHASH_SINGLE || base == SIGHASH_NONE)
        job.flags |= gpu::SIGHASH_JOB_ZERO_SEQUENCE | gpu::SIGHASH_JOB_ZERO_OUTPUTS;
    const COutPoint& op = tx.vin[nIn].prevout;
    memcpy(job.outpoint, op.hash.begin(), 32);
    PutLE32(job.outpoint + 32, op.n);
    const uint64_t a = (uint64_t)amount;
    for (int i = 0; i < 8; ++i) job.amount[i] = (unsigned char)(a >> (8 * i));
    PutLE32(job.sequence, tx.vin[nIn].nSequence);
    return true;
}

uint256 SighashFromRecipe(const gpu::SighashTx& tx, const gpu::SighashJob& job, const unsigned char* code) {
    static const unsigned char zero[32] = {};
    HashWriter ss;
    ss.write((const char*)(tx.version), 4);
    ss.write((const char*)((job.flags & gpu::SIGHASH_JOB_ZERO_PREVOUTS) ? zero : tx.hashPrevouts), 32);
    ss.write((const char*)((job.flags & gpu::SIGHASH_JOB_ZERO_SEQUENCE) ? zero : tx.hashSequence), 32);
    ss.write((const char*)(job.outpoint), 36);
    WriteCompactSize(ss, job.codeLen);
    if (job.codeLen) ss.write((const char*)(code + job.codeOff), job.codeLen);
    ss.write((const char*)(job.amount), 8);
    ss.write((const char*)(job.sequence), 4);
    ss.write((const char*)((job.flags & gpu::SIGHASH_JOB_ZERO_OUTPUTS) ? zero : tx.hashOutputs), 32);
    ss.write((const char*)(tx.lockTime), 4);
    unsigned char ht[4];
    PutLE32(ht, job.hashType);
    ss.write((const char*)(ht), 4);
    return ss.GetHash();
}

} // namespace bcp
