"""Pure-Python P2P test framework for bcpd (functional and conformance tests).

Parity: the reference's test/functional/test_framework/ (mininode.py message classes and
NodeConn, blocktools.py, script.py, comptool.py's accept/reject driver). This package is an
independent implementation of the wire format and of the block-building rules, used as the
oracle the node is tested against:

* ``messages``  - serialization, transactions, the BCP dual-format block header (legacy 80 B
  vs 140 B + Equihash solution), every P2P message the node speaks, BIP152 compact blocks
  (SipHash short ids) and BIP37 bloom filters;
* ``p2p``       - a threaded P2P peer (``P2PPeer``) that can present itself as a current
  (70016) or a legacy (< 70016, 80-byte header) client;
* ``script``    - script builder, opcodes, FORKID signature hashes and signing;
* ``blocktools``- coinbase/transaction/block construction and solving: SHA256d before the
  fork, Equihash (via the node's CPU solver, ``native.eh_solve_cpu``) plus SHA256d after it -
  unlike the reference's Python peer, which can only mine pre-fork blocks;
* ``comparison``- ``BlockRuleDriver``: deliver a block or header, then assert acceptance
  (new tip) or rejection with an exact reject reason.
"""
