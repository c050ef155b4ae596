"""Pure-Python textbook restatement of the reference verify contract.

TEST INFRASTRUCTURE ONLY.  A second, independent restatement (Python big
integers, affine/extended textbook formulas) used to cross-check the C
oracle in oracle/ on the golden vectors.  It follows SURVEY.md Appendix A:

  fd_ed25519_user.c:135-230 (single), :232-310 (batch_single_msg)
  avx512/fd_r43x6_ge.c:163-254 (decode rules; mapping="avx512")
  fd_curve25519.c:22-49 + ref/fd_curve25519.c:209-224 (mapping="ref")
  fd_curve25519.h:84-114 (small order)

Slow (milliseconds per signature): use only on small vector sets.
"""
import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)

SUCCESS, ERR_SIG, ERR_PUBKEY, ERR_MSG = 0, -1, -2, -3


def _inv(x):
    return pow(x, P - 2, P)


def _add(p1, p2):
    # extended coordinates, a = -1 (HWCD add-2008-hwcd-3)
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    B = (Y1 + X1) * (Y2 + X2) % P
    C = T1 * 2 * D * T2 % P
    Dd = Z1 * 2 * Z2 % P
    E, F, G, H = B - A, Dd - C, Dd + C, B + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def _mul(s, p):
    q = (0, 1, 1, 0)
    while s > 0:
        if s & 1:
            q = _add(q, p)
        p = _add(p, p)
        s >>= 1
    return q


def _eq(p1, p2):
    X1, Y1, Z1, _ = p1
    X2, Y2, Z2, _ = p2
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


def decode(enc, mapping="avx512"):
    """Returns the extended point or None (decode failure)."""
    y = int.from_bytes(enc, "little") & ((1 << 255) - 1)
    sign = enc[31] >> 7
    y %= P  # non-canonical y in [p, 2^255) accepted (avx512/fd_f25519.h:100-109)
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    vx2 = v * x * x % P
    if vx2 != u and vx2 != (-u) % P:
        return None
    if vx2 != u:
        x = x * SQRTM1 % P
    if mapping == "avx512" and x == 0 and sign == 1:
        return None
    if (x & 1) != sign:
        x = (-x) % P
    return (x, y, 1, x * y % P)


def _small_order(pt):
    # [8]P == O, evaluated exactly
    return _eq(_mul(8, pt), (0, 1, 1, 0))


B = decode(bytes([0x58] + [0x66] * 31))


def _pass1(msg, sig, pub, mapping):
    r, s = sig[:32], sig[32:]
    S = int.from_bytes(s, "little")
    if S >= L:
        return ERR_SIG, None
    A = decode(pub, mapping)
    if A is None:
        return (ERR_SIG if mapping == "avx512" else ERR_PUBKEY), None
    R = decode(r, mapping)
    if R is None:
        return ERR_SIG, None
    if _small_order(A):
        return ERR_PUBKEY, None
    if _small_order(R):
        return ERR_SIG, None
    k = int.from_bytes(hashlib.sha512(r + pub + msg).digest(), "little") % L
    return SUCCESS, (A, R, S, k)


def _pass2(st):
    A, R, S, k = st
    negA = ((-A[0]) % P, A[1], A[2], (-A[3]) % P)
    Rc = _add(_mul(S, B), _mul(k, negA))
    return SUCCESS if _eq(Rc, R) else ERR_MSG


def verify(msg, sig, pub, mapping="avx512"):
    rc, st = _pass1(msg, sig, pub, mapping)
    if rc:
        return rc
    return _pass2(st)


def verify_batch_single_msg(msg, sigs, pubs, n, mapping="avx512"):
    if n == 0 or n > 16:
        return ERR_SIG
    sts = []
    for j in range(n):
        rc, st = _pass1(msg, sigs[64 * j:64 * j + 64], pubs[32 * j:32 * j + 32], mapping)
        if rc:
            return rc
        sts.append(st)
    for st in sts:
        if _pass2(st):
            return ERR_MSG
    return SUCCESS
