// Node context: the long-lived subsystems of one running node (reference globals
// pcoinsTip/mempool/g_connman/pwalletMain wired up by src/init.cpp AppInitMain).
#pragma once
#include "consensus/params.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "util/util.h"

#include <memory>
#include <string>

namespace bcp {

class CConnman;
class CKeyStore;
class CWallet;
class HTTPServer;
class ZMQNotifier;

struct NodeContext {
    const CChainParams* params = nullptr;
    std::string datadir;
    bool useGpu = true;
    std::unique_ptr<CBlockPolicyEstimator> estimator;
    std::unique_ptr<CTxMemPool> mempool;
    std::unique_ptr<Chainstate> chainstate;
    std::unique_ptr<Scheduler> scheduler;
    CConnman* connman = nullptr;   // owned by init (net layer)
    CWallet* wallet = nullptr;     // owned by init (wallet layer)
    CKeyStore* keystore = nullptr; // wallet key store used by signrawtransaction
    HTTPServer* http = nullptr;
    ZMQNotifier* zmq = nullptr;
};

NodeContext* GetNode();
void SetNode(NodeContext* n);

// Build chainstate + mempool for `chain` in `datadir` (no networking, no RPC server):
// the embedded-node path used by tests and tools.
std::unique_ptr<NodeContext> CreateNode(const std::string& chain, const std::string& datadir, bool memoryOnly,
                                        bool useGpu, std::string& err);
// Construct the subsystems without loading the block index (bcpd drives loading so it
// can -reindex and report warmup progress).
std::unique_ptr<NodeContext> BuildNode(const std::string& chain, const std::string& datadir, bool memoryOnly,
                                       bool wipe, bool useGpu);
void ShutdownNode(NodeContext& node);

} // namespace bcp
