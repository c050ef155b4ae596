"""The CPU oracle against the reference's own golden vectors (CPU only).

Pins oracle/fd_ed25519_oracle.c before it is trusted as the GPU checker:
  - every bool the reference's tests assert (test_ed25519.c:1072-1142,
    test_ed25519_signature_malleability.c, test_verify.c), and
  - the AVX-512 code checksums derived in SURVEY.md §8(c), and
  - SHA-512 CAVP, the sign KAT (test_ed25519.c:881-885), the small-order
    encodings (test_ed25519.c:613-661).
"""
import collections
import hashlib
import random

import numpy as np
import pytest

import pyref_ed25519 as pyref

L = 2**252 + 27742317777372353535851937790883648493


def _codes(vectors, src, key="code"):
    return collections.Counter(v[key] for v in vectors["vectors"] if v["src"] == src)


def test_vector_counts(vectors):
    c = collections.Counter(v["src"] for v in vectors["vectors"])
    assert c == {"cctv": 914, "wycheproof": 133, "malleability_should_fail": 196, "malleability_should_pass": 200}


def test_oracle_reproduces_reference_bools_and_codes(vectors, oracle):
    for v in vectors["vectors"]:
        msg, sig, pub = (bytes.fromhex(v[k]) for k in ("msg", "sig", "pub"))
        code = oracle.verify(msg, sig, pub, oracle.MAP_AVX512)
        assert code == v["code"], (v["src"], v["tc_id"])
        assert (code == 0) == bool(v["ref_ok"]), (v["src"], v["tc_id"])
        code_ref = oracle.verify(msg, sig, pub, oracle.MAP_REF)
        assert code_ref == v["code_refmap"], (v["src"], v["tc_id"])
        assert (code_ref == 0) == bool(v["ref_ok"])


def test_survey_code_checksums(vectors):
    """SURVEY.md §8(c) derived checksums (AVX-512 mapping; ref mapping)."""
    assert _codes(vectors, "cctv") == {0: 43, -1: 442, -2: 366, -3: 63}
    assert _codes(vectors, "cctv", "code_refmap") == {0: 43, -1: 282, -2: 526, -3: 63}
    assert _codes(vectors, "wycheproof") == {0: 84, -1: 36, -3: 13}
    assert _codes(vectors, "malleability_should_fail") == {-2: 121, -1: 75}
    assert _codes(vectors, "malleability_should_pass") == {0: 200}
    diff = sum(v["code"] != v["code_refmap"] for v in vectors["vectors"] if v["src"] == "cctv")
    assert diff == 160


def test_oracle_matches_python_restatement_sample(vectors, oracle):
    rnd = random.Random(7)
    sample = rnd.sample(vectors["vectors"], 120)
    for v in sample:
        msg, sig, pub = (bytes.fromhex(v[k]) for k in ("msg", "sig", "pub"))
        assert pyref.verify(msg, sig, pub, "avx512") == v["code"]
        assert pyref.verify(msg, sig, pub, "ref") == v["code_refmap"]


def test_cctv_batch_semantics(vectors, oracle):
    """test_ed25519.c:1101-1142: adversarial vector at index 1 of a valid batch."""
    b = vectors["cctv_batch"]
    msg, sigs, pubs = (bytes.fromhex(b[k]) for k in ("msg", "sigs", "pubs"))
    cctv = [v for v in vectors["vectors"] if v["src"] == "cctv"]
    assert oracle.verify_batch_single_msg(msg, sigs, pubs, 16) == 0
    assert len(b["cases"]) > 50
    for case in b["cases"]:
        v = cctv[case["cctv_index"]]
        s = bytearray(sigs); p = bytearray(pubs)
        s[64:128] = bytes.fromhex(v["sig"]); p[32:64] = bytes.fromhex(v["pub"])
        assert oracle.verify_batch_single_msg(msg, bytes(s), bytes(p), 2) == case["code2"]
        assert oracle.verify_batch_single_msg(msg, bytes(s), bytes(p), 4) == case["code4"]
        assert (case["code2"] == 0) == bool(case["ref_ok"])


def test_batch_size_limits(oracle):
    """fd_ed25519_user.c:238-241: batch_sz 0 or > 16 -> ERR_SIG."""
    assert oracle.verify_batch_single_msg(b"x", b"\0" * 64, b"\0" * 32, 0) == -1
    assert oracle.verify_batch_single_msg(b"x", b"\0" * 64 * 17, b"\0" * 32 * 17, 17) == -1


def test_first_error_ordering(oracle, misc_vectors):
    """Pass 1 reports a structural error of a LATER signature before an
    equation failure of an earlier one (fd_ed25519_user.c:264-306)."""
    prv = bytes(range(32))
    msg = b"ordering"
    pub = oracle.public_from_private(prv)
    sig = oracle.sign(msg, pub, prv)
    bad_eq = bytearray(sig); bad_eq[40] ^= 1           # S changed: still < L most likely -> ERR_MSG
    bad_s = bytearray(sig); bad_s[63] = 0xff           # S >= L -> ERR_SIG
    assert oracle.verify(msg, bytes(bad_eq), pub) == -3
    assert oracle.verify(msg, bytes(bad_s), pub) == -1
    assert oracle.verify_batch_single_msg(msg, bytes(bad_eq) + bytes(bad_s), pub + pub, 2) == -1
    assert oracle.verify_batch_single_msg(msg, bytes(bad_eq) + sig, pub + pub, 2) == -3
    assert oracle.verify_batch_single_msg(msg, sig + sig, pub + pub, 2) == 0


def test_sign_kat(misc_vectors, oracle):
    k = misc_vectors["sign_kat"]
    prv = bytes.fromhex(k["prv"])
    pub = oracle.public_from_private(prv)
    assert oracle.sign(b"", pub, prv).hex() == k["sig"]


def test_fuzz_corpus_sign_verify(misc_vectors, oracle):
    """corpus/fuzz_ed25519_sigverify: prv||msg, sign then verify succeeds."""
    assert len(misc_vectors["fuzz"]) == 4
    for f in misc_vectors["fuzz"]:
        prv, msg = bytes.fromhex(f["prv"]), bytes.fromhex(f["msg"])
        pub = oracle.public_from_private(prv)
        assert pub.hex() == f["pub"]
        sig = oracle.sign(msg, pub, prv)
        assert sig.hex() == f["sig"]
        assert oracle.verify(msg, sig, pub) == 0


def test_small_order_encodings(misc_vectors, oracle):
    """test_ed25519.c:613-661 (frombytes + affine_is_small_order)."""
    for e in misc_vectors["small_order"]:
        rc, so, _ = oracle.point_decode(bytes.fromhex(e["enc"]), oracle.MAP_REF)
        if rc == 0:
            assert so == e["small_order"], e
        else:
            assert e["small_order"] == 0, e   # failed decode leaves the point non-small in the test


def test_sha512_cavp(sha_vectors, oracle):
    for v in sha_vectors["short"] + sha_vectors["long"]:
        assert oracle.sha512(bytes.fromhex(v["msg"])).hex() == v["md"]
    # Monte Carlo (SHA512Monte.rsp): MD_i = SHA(MD_{i-3} || MD_{i-2} || MD_{i-1})
    seed = bytes.fromhex(sha_vectors["monte"]["seed"])
    for j, exp in enumerate(sha_vectors["monte"]["md"][:10]):
        md = [seed, seed, seed]
        for _ in range(1000):
            md = [md[1], md[2], oracle.sha512(md[0] + md[1] + md[2])]
        seed = md[2]
        assert seed.hex() == exp, j


def test_scalar_reduce_and_validate(oracle):
    rnd = random.Random(3)
    for x in [0, 1, L - 1, L, L + 1, 2**252, 2**512 - 1, L * L, (L - 1) * 2**256] + [rnd.getrandbits(512) for _ in range(500)]:
        x %= 2**512
        assert int.from_bytes(oracle.scalar_reduce(x.to_bytes(64, "little")), "little") == x % L
    for s, ok in [(0, 1), (1, 1), (L - 1, 1), (L, 0), (L + 1, 0), (2**253 - 1, 0), (2**256 - 1, 0)]:
        assert oracle.scalar_validate(s.to_bytes(32, "little")) == bool(ok)


def test_txn_fixtures(txn_fixtures, oracle):
    """transaction{1..6}.bin and test_verify.c's five hex transactions."""
    by = {t["name"]: t for t in txn_fixtures}
    assert by["test_verify.valid_txn_1sig"]["code"] == 0
    assert by["test_verify.valid_txn_2sigs"]["code"] == 0
    assert by["test_verify.invalid_txn_2sigs"]["code"] != 0
    assert by["test_verify.invalid_txn_same_1sig"]["code"] != 0
    assert by["test_verify.invalid_txn_1sig_same_64bit"]["code"] != 0
    assert [by[f"transaction{i}"]["code"] for i in range(1, 7)] == [0, 0, -1, 0, -1, 0]
    for t in txn_fixtures:
        p = bytes.fromhex(t["payload"])
        n = t["sig_cnt"]
        code = oracle.verify_batch_single_msg(p[t["msg_off"]:], p[1:1 + 64 * n],
                                              p[t["pub_off"]:t["pub_off"] + 32 * n], n)
        assert code == t["code"], t["name"]


def test_quic_corpus_all_valid(quic_corpus, oracle):
    arena, txns, codes = quic_corpus
    assert len(txns) == 1000 and int(txns["sig_cnt"].sum()) == 1006
    sub = txns[:200]
    assert (oracle.verify_txns(arena, sub) == 0).all()
    assert (codes == 0).all()


def test_signer_matches_hashlib_based_pyref(oracle):
    prv = hashlib.sha256(b"k").digest()
    pub = oracle.public_from_private(prv)
    sig = oracle.sign(b"hello", pub, prv)
    assert pyref.verify(b"hello", sig, pub) == 0
