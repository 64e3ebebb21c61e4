// Import of the reference's Berkeley DB wallet.dat without libdb.
//
// The reference keeps the wallet in a BDB 4.8 btree file (src/wallet/db.h:26 CDBEnv,
// src/wallet/walletdb.cpp CWalletDB): a master database whose sub-database "main" holds every
// record, keyed and valued exactly as this wallet's store keys and values them (a serialized type
// string plus key, the serialized value). Importing is therefore copying the records: these
// readers recover them either from the file itself (meta page, internal and leaf btree pages,
// overflow chains; little-endian files without checksums or encryption, as the reference
// writes them) or from the text form that `db_dump` and the reference's salvage produce
// (src/wallet/db.cpp:170-230: HEADER=END, then hex key / hex value lines, DATA=END).
#pragma once
#include <istream>
#include <string>
#include <utility>
#include <vector>

namespace bcp {

using BdbRecords = std::vector<std::pair<std::string, std::string>>;

// What is at `path`: a regular file that is a BDB btree ("btree"), db_dump text ("dump") or
// neither ("").
std::string BdbFileKind(const std::string& path);
// Every live record of the btree file at `path` (sub-database "main" when the file has
// sub-databases, else the master database), in key order.
bool ReadBdbBtree(const std::string& path, BdbRecords& out, std::string& err);
// The records of db_dump's "bytevalue" text format.
bool ReadBdbDump(std::istream& in, BdbRecords& out, std::string& err);

} // namespace bcp

namespace bcp {
// Converts a reference wallet at `path` (a BDB btree file or db_dump text) into this wallet's
// store at the same path: the file is renamed to <path>.bdb.<time>, and every record is written
// to a fresh store unchanged. `imported` receives the record count.
bool ImportBdbWalletFile(const std::string& path, size_t& imported, std::string& err);
} // namespace bcp
