#!/usr/bin/env python3
"""Create an -rpcauth line for bcp.conf: the node stores a salted HMAC of the password, not the
password itself.

    share/rpcauth/rpcauth.py <username> [<password>]

Prints `rpcauth=<username>:<salt>$<hmac>` for the config file and the password to give the RPC
client. A random 32-byte password is generated if none is given. The HMAC is
HMAC-SHA256(key=salt, message=password), hex-encoded, which is what bcpd checks
(csrc/rpc/httpserver.cpp).

Parity: reference share/rpcauth/rpcauth.py (same line format and HMAC).
"""
import base64
import hmac
import os
import sys


def generate_salt(size: int = 16) -> str:
    return os.urandom(size).hex()


def generate_password() -> str:
    return base64.urlsafe_b64encode(os.urandom(32)).decode("utf-8")


def password_to_hmac(salt: str, password: str) -> str:
    return hmac.new(salt.encode("utf-8"), password.encode("utf-8"), "SHA256").hexdigest()


def main(argv):
    if not 1 <= len(argv) <= 2:
        print(__doc__.strip(), file=sys.stderr)
        return 1
    user = argv[0]
    password = argv[1] if len(argv) == 2 else generate_password()
    salt = generate_salt()
    print("String to be appended to bcp.conf:")
    print(f"rpcauth={user}:{salt}${password_to_hmac(salt, password)}")
    print(f"Your password:\n{password}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
