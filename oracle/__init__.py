"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- see fd_ed25519_oracle.c."""
