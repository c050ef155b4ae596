"""The engine process's command line (firedancer_amd/engine_proc.py main) for
the CPU tests: the same gather-mode verify mux tiles over shared-memory
links, with the test's checker -- the CPU oracle behind a host stand-in of
the engine's gathered-batch calls (tile.PyVerifier: each payload read late,
at the poll that completes its batch, its in-mcache line re-checked after
the read) -- in place of the GPU engines.  tools/xproc.py runs it as
`python tests/_engine_proc_worker.py <engine_proc arguments>`."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def oracle_verifiers(T, a):
    from firedancer_amd import tile
    from oracle import oracle as orc
    orc.lib()                       # loaded before the process enters its sandbox (--sandbox)
    vers = [tile.PyVerifier(lambda arena, txns: orc.verify_txns(arena, txns), slots=a.inflight, lag=1)
            for _ in range(T)]
    return vers, (lambda: None), {"device": None, "verifier": "oracle (test stand-in)"}


if __name__ == "__main__":
    from firedancer_amd import engine_proc
    sys.exit(engine_proc.main(sys.argv[1:], make_verifiers=oracle_verifiers))
