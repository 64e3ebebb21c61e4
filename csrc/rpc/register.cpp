#include "rpc/server.h"

namespace bcp {

// Optional groups provide weak defaults so a build without them still links.
__attribute__((weak)) void RegisterNetRPCCommands(CRPCTable&) {}
__attribute__((weak)) void RegisterWalletRPCCommands(CRPCTable&) {}

void RegisterAllRPCCommands(CRPCTable& t) {
    static bool done = false;
    if (done) return;
    done = true;
    RegisterBlockchainRPCCommands(t);
    RegisterMiningRPCCommands(t);
    RegisterRawTransactionRPCCommands(t);
    RegisterMiscRPCCommands(t);
    RegisterABCRPCCommands(t);
    RegisterNetRPCCommands(t);
    RegisterWalletRPCCommands(t);
}

} // namespace bcp
