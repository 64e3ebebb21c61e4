// merkle_tests: BlockMerkleRoot / BlockMerkleBranch / ComputeMerkleRootFromBranch against a
// straightforward whole-tree builder, for blocks of 0..16 and random larger sizes, each also
// mutated by duplicating its last 1-3 power-of-two runs of transactions (CVE-2012-2459): the
// root stays the same and the mutation flag is raised.
// Parity: reference src/test/merkle_tests.cpp (merkle_test, with its BlockBuildMerkleTree and
// BlockGetMerkleBranch reference implementations).
#include "test/unittest.h"

#include "consensus/merkle.h"
#include "primitives/serialize.h"

#include <algorithm>

using namespace bcp;

namespace {

// every level of the tree, leaves first (the original satoshi-client construction)
uint256 BuildTree(const CBlock& block, bool* fMutated, std::vector<uint256>& tree) {
    tree.clear();
    for (const auto& tx : block.vtx) tree.push_back(tx->GetHash());
    size_t j = 0;
    bool mutated = false;
    for (int nSize = (int)block.vtx.size(); nSize > 1; nSize = (nSize + 1) / 2) {
        for (int i = 0; i < nSize; i += 2) {
            const int i2 = std::min(i + 1, nSize - 1);
            if (i2 == i + 1 && i2 + 1 == nSize && tree[j + i] == tree[j + i2]) mutated = true;
            tree.push_back(Hash256Concat(tree[j + i], tree[j + i2]));
        }
        j += nSize;
    }
    if (fMutated) *fMutated = mutated;
    return tree.empty() ? uint256() : tree.back();
}

std::vector<uint256> TreeBranch(const CBlock& block, const std::vector<uint256>& tree, int nIndex) {
    std::vector<uint256> branch;
    size_t j = 0;
    for (int nSize = (int)block.vtx.size(); nSize > 1; nSize = (nSize + 1) / 2) {
        const int i = std::min(nIndex ^ 1, nSize - 1);
        branch.push_back(tree[j + i]);
        nIndex >>= 1;
        j += nSize;
    }
    return branch;
}

int ctz(uint32_t i) {
    if (i == 0) return 0;
    int j = 0;
    while (!(i & 1)) {
        j++;
        i >>= 1;
    }
    return j;
}

} // namespace

TEST_CASE(merkle_tests, merkle_test) {
    FastRandomContext rng(true);
    for (int i = 0; i < 32; i++) {
        // every size 0..16, then 15 random sizes
        const int ntx = i <= 16 ? i : 17 + (int)rng.randrange(4000);
        for (int mutate = 0; mutate <= 3; mutate++) {
            // duplicate the last 2^ctz(n) transactions, up to three times
            const int dup1 = mutate >= 1 ? 1 << ctz(ntx) : 0;
            if (dup1 >= ntx) break; // duplicating the whole tree adds a level: a different root
            const int ntx1 = ntx + dup1;
            const int dup2 = mutate >= 2 ? 1 << ctz(ntx1) : 0;
            if (dup2 >= ntx1) break;
            const int ntx2 = ntx1 + dup2;
            const int dup3 = mutate >= 3 ? 1 << ctz(ntx2) : 0;
            if (dup3 >= ntx2) break;
            const int ntx3 = ntx2 + dup3;

            CBlock block;
            block.vtx.resize(ntx);
            for (int j = 0; j < ntx; j++) {
                CMutableTransaction mtx;
                mtx.nLockTime = (uint32_t)j;
                block.vtx[j] = MakeTransactionRef(std::move(mtx));
            }
            bool unmutatedMutated = false;
            const uint256 unmutatedRoot = BlockMerkleRoot(block, &unmutatedMutated);
            CHECK(!unmutatedMutated);

            block.vtx.resize(ntx3);
            for (int j = 0; j < dup1; j++) block.vtx[ntx + j] = block.vtx[ntx + j - dup1];
            for (int j = 0; j < dup2; j++) block.vtx[ntx1 + j] = block.vtx[ntx1 + j - dup2];
            for (int j = 0; j < dup3; j++) block.vtx[ntx2 + j] = block.vtx[ntx2 + j - dup3];

            bool oldMutated = false;
            std::vector<uint256> tree;
            const uint256 oldRoot = BuildTree(block, &oldMutated, tree);
            bool newMutated = false;
            const uint256 newRoot = BlockMerkleRoot(block, &newMutated);
            CHECK(oldRoot == newRoot);
            CHECK(newRoot == unmutatedRoot);
            CHECK((newRoot == uint256()) == (ntx == 0));
            CHECK_EQ(oldMutated, newMutated);
            CHECK_EQ(newMutated, mutate != 0);
            if (mutate == 0) { // branches: all of them up to 16 transactions, else 16 random ones
                for (int loop = 0; loop < std::min(ntx, 16); loop++) {
                    const int m = ntx > 16 ? (int)rng.randrange(ntx) : loop;
                    const std::vector<uint256> newBranch = BlockMerkleBranch(block, (uint32_t)m);
                    const std::vector<uint256> oldBranch = TreeBranch(block, tree, m);
                    CHECK(oldBranch == newBranch);
                    CHECK(ComputeMerkleRootFromBranch(block.vtx[m]->GetHash(), newBranch, (uint32_t)m) == oldRoot);
                }
            }
        }
    }
}
