"""Generate the committed golden fixtures under tests/golden/ from the
reference's own test data.

Runs ONLY in the build container (it reads /root/reference as TEXT/DATA;
nothing of the reference is compiled, imported or executed).  The outputs
are committed; the GPU box never sees /root/reference.

Sources (all parsed as text or raw bytes):
  src/ballet/ed25519/test_ed25519_cctv.c            914 vectors, bool `ok`
  src/ballet/ed25519/test_ed25519_wycheproof.c      133 vectors, bool `ok`
  src/ballet/ed25519/test_ed25519_signature_malleability_should_{fail,pass}.bin
                                                    96-B records sig||pub, msg "Zcash"
                                                    (test_ed25519_signature_malleability.c:16-50)
  src/ballet/ed25519/test_ed25519.c:604-711         small-order / validate encodings
  src/ballet/ed25519/test_ed25519.c:881-885         sign KAT (prv, empty msg, sig)
  src/ballet/txn/fixtures/transaction{1..6}.bin     raw txns
  src/app/fdctl/run/tiles/test_verify.c:4-105       5 hex txns (tile-level test)
  src/waltz/quic/tests/txn/tx                       1000 base64 txns
  corpus/fuzz_ed25519_sigverify/*                   prv[32]||msg (fuzz_ed25519_sigverify.c:23-50)
  src/ballet/sha512/cavp/SHA512{Short,Long}Msg.rsp, SHA512Monte.rsp

Expected result codes are computed with the C oracle (oracle/liboracle.so)
and cross-checked against the pure-Python restatement (tests/pyref_ed25519.py)
and against every bool the reference's tests assert.
"""
import base64
import glob
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from oracle import oracle as orc  # noqa: E402
import pyref_ed25519 as pyref  # noqa: E402


def c_str_bytes(s):
    """Decode a C string literal body made of \\xNN escapes and plain chars."""
    out = bytearray()
    i = 0
    while i < len(s):
        if s[i] == "\\":
            if s[i + 1] == "x":
                out.append(int(s[i + 2:i + 4], 16))
                i += 4
                continue
            esc = {"n": 10, "t": 9, "r": 13, "0": 0, "\\": 92, '"': 34}
            out.append(esc[s[i + 1]])
            i += 2
        else:
            out.append(ord(s[i]))
            i += 1
    return bytes(out)


ENTRY_RE = re.compile(
    r"\{\s*\.tc_id\s*=\s*(\d+),\s*\.comment\s*=\s*\"((?:[^\"\\]|\\.)*)\",\s*"
    r"\.msg\s*=\s*\(uchar const \*\)\"((?:[^\"\\]|\\.)*)\",\s*\.msg_sz\s*=\s*(\d+)UL,\s*"
    r"\.sig\s*=\s*\"((?:[^\"\\]|\\.)*)\",\s*\.pub\s*=\s*\"((?:[^\"\\]|\\.)*)\",\s*\.ok\s*=\s*(\d)\s*\}",
    re.S)


def parse_vector_file(path, src):
    text = open(path).read()
    out = []
    for m in ENTRY_RE.finditer(text):
        tc_id, comment, msg, msg_sz, sig, pub, ok = m.groups()
        msg = c_str_bytes(msg)
        assert len(msg) == int(msg_sz), (src, tc_id)
        sig, pub = c_str_bytes(sig), c_str_bytes(pub)
        assert len(sig) == 64 and len(pub) == 32
        out.append(dict(src=src, tc_id=int(tc_id), comment=c_str_bytes(comment).decode("latin1"),
                        msg=msg.hex(), sig=sig.hex(), pub=pub.hex(), ref_ok=int(ok)))
    return out


def compact_u16(b, i):
    v = 0
    for k in range(3):
        byte = b[i + k]
        v |= (byte & 0x7F) << (7 * k)
        if not byte & 0x80:
            return v, k + 1
    raise ValueError("bad compact-u16")


def parse_txn_offsets(p):
    """Minimal restatement of fd_txn_parse_core offsets (fd_txn_parse.c:79-134)."""
    n = p[0]
    sig_off = 1
    msg_off = 1 + 64 * n
    i = msg_off
    if p[i] & 0x80:
        i += 2  # version byte, then sig_cnt copy
    else:
        i += 1
    i += 2  # ro_signed, ro_unsigned
    acct_cnt, used = compact_u16(p, i)
    i += used
    return dict(sig_cnt=n, sig_off=sig_off, pub_off=i, msg_off=msg_off, acct_cnt=acct_cnt)


def hex_txn(lines):
    return bytes.fromhex("".join(lines))


def parse_test_verify_txns():
    text = open(f"{REF}/src/app/fdctl/run/tiles/test_verify.c").read()
    out = {}
    for m in re.finditer(r"static char \*\s*\n(\w+)\[\] = \{(.*?)\};", text, re.S):
        name, body = m.groups()
        parts = re.findall(r"\"([0-9a-f]*)\"", body)
        out[name] = hex_txn(parts)
    return out


def parse_rsp(path):
    vecs, cur = [], {}
    for line in open(path):
        line = line.strip()
        if line.startswith("Len ="):
            cur = {"len": int(line.split("=")[1])}
        elif line.startswith("Msg =") and cur:
            cur["msg"] = line.split("=")[1].strip()
        elif line.startswith("MD =") and "len" in cur:
            cur["md"] = line.split("=")[1].strip()
            nbytes = cur["len"] // 8
            vecs.append(dict(msg=cur["msg"][:2 * nbytes], md=cur["md"]))
            cur = {}
    return vecs


def parse_monte(path):
    seed, mds = None, []
    for line in open(path):
        line = line.strip()
        if line.startswith("Seed ="):
            seed = line.split("=")[1].strip()
        elif line.startswith("MD ="):
            mds.append(line.split("=")[1].strip())
    return dict(seed=seed, md=mds)


def main():
    ed = []
    ed += parse_vector_file(f"{REF}/src/ballet/ed25519/test_ed25519_cctv.c", "cctv")
    ed += parse_vector_file(f"{REF}/src/ballet/ed25519/test_ed25519_wycheproof.c", "wycheproof")
    n_cctv = sum(v["src"] == "cctv" for v in ed)
    n_wy = sum(v["src"] == "wycheproof" for v in ed)
    assert (n_cctv, n_wy) == (914, 133), (n_cctv, n_wy)
    for name, ok in (("should_fail", 0), ("should_pass", 1)):
        raw = open(f"{REF}/src/ballet/ed25519/test_ed25519_signature_malleability_{name}.bin", "rb").read()
        assert len(raw) % 96 == 0
        for i in range(len(raw) // 96):
            rec = raw[96 * i:96 * i + 96]
            ed.append(dict(src="malleability_" + name, tc_id=i, comment="", msg=b"Zcash".hex(),
                           sig=rec[:64].hex(), pub=rec[64:].hex(), ref_ok=ok))

    # expected codes: C oracle, cross-checked with the Python restatement
    mism = 0
    for v in ed:
        msg, sig, pub = bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"])
        v["code"] = orc.verify(msg, sig, pub, orc.MAP_AVX512)
        v["code_refmap"] = orc.verify(msg, sig, pub, orc.MAP_REF)
        py = pyref.verify(msg, sig, pub, "avx512")
        pyr = pyref.verify(msg, sig, pub, "ref")
        if py != v["code"] or pyr != v["code_refmap"]:
            mism += 1
            print("ORACLE/PYREF MISMATCH", v["src"], v["tc_id"], v["code"], py, v["code_refmap"], pyr)
        if (v["code"] == 0) != bool(v["ref_ok"]) or (v["code_refmap"] == 0) != bool(v["ref_ok"]):
            mism += 1
            print("REFERENCE BOOL MISMATCH", v["src"], v["tc_id"], v["ref_ok"], v["code"], v["code_refmap"])
    assert mism == 0, mism

    # cctv batch semantics (test_ed25519.c:1101-1142): msg of cctvs[7]; 16 valid
    # signatures over it from the oracle signer, vector placed at index 1.
    cctv = [v for v in ed if v["src"] == "cctv"]
    bmsg = bytes.fromhex(cctv[7]["msg"])
    rng = np.random.default_rng(0x5EED0C7)
    bsigs, bpubs = bytearray(), bytearray()
    for j in range(16):
        prv = rng.bytes(32)
        pub = orc.public_from_private(prv)
        bsigs += orc.sign(bmsg, pub, prv)
        bpubs += pub
    batch = dict(msg=bmsg.hex(), sigs=bytes(bsigs).hex(), pubs=bytes(bpubs).hex(), cases=[])
    assert orc.verify_batch_single_msg(bmsg, bytes(bsigs), bytes(bpubs), 16) == 0
    for idx, v in enumerate(cctv):
        if v["msg"] != cctv[7]["msg"]:
            continue
        s, p = bytearray(bsigs), bytearray(bpubs)
        s[64:128] = bytes.fromhex(v["sig"])
        p[32:64] = bytes.fromhex(v["pub"])
        c2 = orc.verify_batch_single_msg(bmsg, bytes(s[:128]), bytes(p[:64]), 2)
        c4 = orc.verify_batch_single_msg(bmsg, bytes(s[:256]), bytes(p[:128]), 4)
        assert (c2 == 0) == bool(v["ref_ok"]) and (c4 == 0) == bool(v["ref_ok"])
        assert pyref.verify_batch_single_msg(bmsg, bytes(s[:256]), bytes(p[:128]), 4) == c4
        batch["cases"].append(dict(cctv_index=idx, tc_id=v["tc_id"], code2=c2, code4=c4, ref_ok=v["ref_ok"]))

    # txn fixtures
    txns = []
    for k in range(1, 7):
        p = open(f"{REF}/src/ballet/txn/fixtures/transaction{k}.bin", "rb").read()
        txns.append(dict(name=f"transaction{k}", payload=p.hex(), **parse_txn_offsets(p)))
    for name, p in parse_test_verify_txns().items():
        txns.append(dict(name=f"test_verify.{name}", payload=p.hex(), **parse_txn_offsets(p)))
    for t in txns:
        p = bytes.fromhex(t["payload"])
        n = t["sig_cnt"]
        t["code"] = orc.verify_batch_single_msg(p[t["msg_off"]:], p[1:1 + 64 * n],
                                                p[t["pub_off"]:t["pub_off"] + 32 * n], n)
        t["sig_codes"] = [orc.verify(p[t["msg_off"]:], p[1 + 64 * j:65 + 64 * j],
                                     p[t["pub_off"] + 32 * j:t["pub_off"] + 32 * j + 32]) for j in range(n)]
    exp = {"test_verify.valid_txn_1sig": 0, "test_verify.valid_txn_2sigs": 0,
           "test_verify.invalid_txn_2sigs": -1, "test_verify.invalid_txn_same_1sig": -3,
           "test_verify.invalid_txn_1sig_same_64bit": None}
    for t in txns:
        if t["name"] in exp and exp[t["name"]] is not None:
            assert (t["code"] == 0) == (exp[t["name"]] == 0), t["name"]
        if t["name"] == "test_verify.invalid_txn_1sig_same_64bit":
            assert t["code"] != 0

    # QUIC corpus: 1000 base64 txns -> arena + offsets (binary npz)
    lines = [ln.strip() for ln in open(f"{REF}/src/waltz/quic/tests/txn/tx") if ln.strip()]
    arena, recs, codes = bytearray(), [], []
    for ln in lines:
        p = base64.b64decode(ln)
        off = len(arena)
        arena += p
        o = parse_txn_offsets(p)
        recs.append((off + o["msg_off"], len(p) - o["msg_off"], off + o["sig_off"], off + o["pub_off"], o["sig_cnt"]))
    txn_arr = np.array(recs, dtype=orc.TXN_DTYPE)
    arena_np = np.frombuffer(bytes(arena), dtype=np.uint8)
    qcodes = orc.verify_txns(arena_np, txn_arr, nthreads=8)
    assert (qcodes == 0).all(), np.unique(qcodes, return_counts=True)
    np.savez_compressed(os.path.join(HERE, "quic_txns.npz"), arena=arena_np, txns=txn_arr, codes=qcodes)

    # fuzz corpus: prv || msg -> sign -> verify must succeed
    fuzz = []
    for path in sorted(glob.glob(f"{REF}/corpus/fuzz_ed25519_sigverify/*")):
        raw = open(path, "rb").read()
        if len(raw) < 32:
            continue
        prv, msg = raw[:32], raw[32:]
        pub = orc.public_from_private(prv)
        sig = orc.sign(msg, pub, prv)
        assert orc.verify(msg, sig, pub) == 0
        fuzz.append(dict(name=os.path.basename(path), prv=prv.hex(), msg=msg.hex(), pub=pub.hex(), sig=sig.hex()))

    # encodings from test_ed25519.c (small order: :613-661; validate: :673-711)
    t = open(f"{REF}/src/ballet/ed25519/test_ed25519.c").read()
    so_block = t[t.index("test_affine_is_small_order"):t.index("test_point_validate")]
    small = []
    for m in re.finditer(r"fd_hex_decode\(s, \"([0-9a-f]{64})\", 32 \);\s*fd_ed25519_point_frombytes\( r, s \);\s*FD_TEST\( (!?) ?fd_ed25519_affine_is_small_order", so_block):
        small.append(dict(enc=m.group(1), small_order=0 if m.group(2) == "!" else 1))
    assert len(small) == 10, len(small)
    val_block = t[t.index("test_point_validate"):t.index("test_sc_validate")]
    validate = []
    for m in re.finditer(r"fd_hex_decode\( buf, \"([0-9a-f]{64})\", 32 \);\s*FD_TEST_CUSTOM\( (!?)fd_ed25519_point_validate", val_block):
        validate.append(dict(enc=m.group(1), valid=0 if m.group(2) == "!" else 1))
    assert len(validate) == 11, len(validate)
    sign_kat = dict(prv="57835dc6a20e4efd70e90882dbd832b577dbc469960284e0ee718fb526d2ec84", msg="",
                    sig="d65759870ce42b34fd955871f0371ce1c9a976edbe98417b84541bb4c68b65a0"
                        "673799895c61d530624ffbf92c047d47d4eb4cd1bac2ecee1365faebb53a6303")
    assert sign_kat["prv"] in t and sign_kat["sig"] in t

    # SHA-512 CAVP
    short = parse_rsp(f"{REF}/src/ballet/sha512/cavp/SHA512ShortMsg.rsp")
    long_ = parse_rsp(f"{REF}/src/ballet/sha512/cavp/SHA512LongMsg.rsp")
    monte = parse_monte(f"{REF}/src/ballet/sha512/cavp/SHA512Monte.rsp")
    for v in short + long_:
        assert orc.sha512(bytes.fromhex(v["msg"])).hex() == v["md"]
    sha = dict(short=short, long=long_[::4], monte=monte)

    summary = {}
    for v in ed:
        summary.setdefault(v["src"], {}).setdefault(str(v["code"]), 0)
        summary[v["src"]][str(v["code"])] += 1
    print(json.dumps(summary, indent=1))

    json.dump(dict(vectors=ed, cctv_batch=batch, summary=summary), open(os.path.join(HERE, "ed25519_vectors.json"), "w"))
    json.dump(dict(txns=txns), open(os.path.join(HERE, "txn_fixtures.json"), "w"), indent=1)
    json.dump(dict(fuzz=fuzz, small_order=small, point_validate=validate, sign_kat=sign_kat),
              open(os.path.join(HERE, "misc_vectors.json"), "w"), indent=1)
    json.dump(sha, open(os.path.join(HERE, "sha512_cavp.json"), "w"))
    print("ok", len(ed), "vectors;", len(txns), "txn fixtures;", len(lines), "quic txns;", len(fuzz), "fuzz")


if __name__ == "__main__":
    main()
