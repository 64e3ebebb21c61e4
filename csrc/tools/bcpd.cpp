// bcpd: the Bitcoin Cash Plus daemon (reference src/bitcoind.cpp).
#include "node/init.h"

int main(int argc, char* argv[]) { return bcp::AppMain(argc, argv); }
