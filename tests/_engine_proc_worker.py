"""Spawned-process target for tests/test_engine_proc.py: the engine process
(firedancer_amd.engine_proc.serve) over shared-memory links, with the CPU
oracle as the test's verifier (CPU test) or the GPU engine (GPU test)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(in_path, out_path, frag_cnt, use_gpu, result_q, tile_kw):
    try:
        from firedancer_amd import engine_proc, tile
        if use_gpu:
            from firedancer_amd import VerifyEngine
            eng = VerifyEngine(0, max_txn=4096, max_sig=4096 * 12, max_arena=4096 * 1232, ring_depth=3)
            ver = tile.EngineVerifier([eng])
        else:
            from oracle import oracle as orc
            ver = tile.PyVerifier(lambda arena, txns: orc.verify_txns(arena, txns), slots=3, lag=1)
        st = engine_proc.serve(in_path, out_path, ver, frag_cnt, timeout_s=90.0, **tile_kw)
        if use_gpu:
            ver.close()
            eng.close()
        result_q.put(("ok", st))
    except BaseException as e:          # report, never hang the parent
        result_q.put(("err", repr(e)))
