"""Scala-literal restatement of the reference hash-overlap path -- TEST INFRASTRUCTURE.

This file is part of the oracle (see oracle/README.md): only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() may use it, and only as a checker.

It is a deliberately naive, line-by-line transliteration of the Scala code into
pure Python (small inputs only: crp177-sized).  It exists to cross-check the C
restatement (oracle/sa_oracle.c), which is written for speed.  Every function
cites the reference line it follows (paths relative to /root/reference).

Float32 semantics: all `Float` arithmetic of the reference is reproduced with
numpy.float32 scalars (same IEEE-754 single rounding as the JVM on x86-64).
"""
import bisect
import json
import os

import numpy as np

F32 = np.float32
_PRIMES = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "tests", "golden", "trove_primes.json")))["sorted"]


def i32(x):
    """Wrap to a Java Int."""
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


# --------------------------------------------------------------------------
# GNU Trove 3.0.3 TIntObjectHashMap (lib/trove.jar, bytecode read as data;
# SURVEY.md E1).  Only the operations the reference uses.
# --------------------------------------------------------------------------
def next_prime(desired):  # PrimeFinder.nextPrime: Arrays.binarySearch + insertion point
    return _PRIMES[bisect.bisect_left(_PRIMES, desired)]


class TroveIntMap:
    FREE, FULL = 0, 1

    def __init__(self):  # THash(): THash(10, 0.5f) -> setUp(fastCeil(10/0.5f)=20)
        self.load = F32(0.5)
        cap = next_prime(20)
        self._alloc(cap)
        self.size = 0
        self._compute_max_size(cap)

    def _alloc(self, cap):
        self.keys = [0] * cap
        self.vals = [None] * cap
        self.states = [0] * cap

    def _compute_max_size(self, cap):  # THash.computeMaxSize
        self.max_size = min(cap - 1, int(F32(cap) * self.load))
        self.free = cap - self.size

    def _insert_key(self, val):  # TIntHash.insertKey / insertKeyRehash
        length = len(self.states)
        h = val & 0x7FFFFFFF
        index = h % length
        self.consume_free = False
        if self.states[index] == self.FREE:
            self.consume_free = True
            self.keys[index] = val
            self.states[index] = self.FULL
            return index
        if self.keys[index] == val:
            return -index - 1
        probe = 1 + (h % (length - 2))
        loop = index
        while True:
            index -= probe
            if index < 0:
                index += length
            if self.states[index] == self.FREE:
                self.consume_free = True
                self.keys[index] = val
                self.states[index] = self.FULL
                return index
            if self.keys[index] == val:
                return -index - 1
            if index == loop:
                raise RuntimeError("Trove: table full")

    def _index(self, val):
        length = len(self.states)
        h = val & 0x7FFFFFFF
        index = h % length
        if self.states[index] == self.FREE:
            return -1
        if self.keys[index] == val:
            return index
        probe = 1 + (h % (length - 2))
        loop = index
        while True:
            index -= probe
            if index < 0:
                index += length
            if self.states[index] == self.FREE:
                return -1
            if self.keys[index] == val:
                return index
            if index == loop:
                return -1

    def contains(self, key):
        return self._index(key) >= 0

    def get(self, key):
        i = self._index(key)
        return None if i < 0 else self.vals[i]

    def put(self, key, value):  # TIntObjectHashMap.put / doPut / THash.postInsertHook
        index = self._insert_key(key)
        if index < 0:
            self.vals[-index - 1] = value
            return
        self.vals[index] = value
        if self.consume_free:
            self.free -= 1
        self.size += 1
        if self.size > self.max_size or self.free == 0:
            cap = len(self.states)
            newcap = next_prime(cap << 1) if self.size > self.max_size else cap
            self._rehash(newcap)
            self._compute_max_size(len(self.states))

    def _rehash(self, newcap):  # TIntObjectHashMap.rehash: old slots high -> low
        ok, ov, os_ = self.keys, self.vals, self.states
        self._alloc(newcap)
        for i in range(len(os_) - 1, -1, -1):
            if os_[i] == self.FULL:
                idx = self._insert_key(ok[i])
                self.vals[idx] = ov[i]

    def items(self):  # THashPrimitiveIterator: slots cap-1 .. 0
        for i in range(len(self.states) - 1, -1, -1):
            if self.states[i] == self.FULL:
                yield self.keys[i], self.vals[i]


# --------------------------------------------------------------------------
# ObjectStore.scala
# --------------------------------------------------------------------------
class AlignSettings:  # ObjectStore.scala:17-36, defaults Project4.scala:104-114
    def __init__(self, k=12, gap_open=-200, gap_extend=-20, min_overlap=40,
                 min_identity=0.98, max_ignore=90, min_coll=7, max_coll=222,
                 edge=0.4, center=0.4, cost=None):
        self.kmerSize = k
        self.gapOpen = gap_open
        self.gapExtend = gap_extend
        self.minOverlap = min_overlap
        self.minIdentity = F32(min_identity)
        self.maxIgnore = F32(max_ignore)
        self.minCollisions = min_coll
        self.maxCollisions = max_coll
        e, c = F32(edge), F32(center)
        self.kmerHeadEdge = e
        self.kmerTailEdge = F32(1.0) - e
        self.kmerMidLeadEdge = F32(0.5) - (c * F32(0.5))
        self.kmerMidTailEdge = F32(0.5) + (c * F32(0.5))
        self.cost = cost or default_hoxd_table()


def seq_hash(seq):  # Kmer.seqHash, ObjectStore.scala:48-67
    h = 0
    for i in range(min(16, len(seq))):
        c = seq[i].upper()
        h = i32(h << 2)
        code = {"A": 0, "C": 1, "T": 2, "G": 3}.get(c)
        if code is not None:
            h ^= code
    return h


class Kmer:  # ObjectStore.scala:40-45
    __slots__ = ("int", "id", "loc")

    def __init__(self, i, km, loc):
        self.int = seq_hash(km)
        self.id = i
        self.loc = loc


class Alignment:  # ObjectStore.scala:89-107
    def __init__(self, lenA, lenB, idA, idB, start, end, c, e):
        self.lenA, self.lenB, self.idA, self.idB = lenA, lenB, idA, idB
        self.start, self.end, self.correct, self.error = start, end, c, e
        self.alen = c + e  # alignA.length: one char per backtrack step
        self.errRatio = F32(c) / (F32(c) + F32(e))

    def valid(self, s):
        return (bool(self.errRatio >= s.minIdentity) and self.alen >= s.minOverlap and
                ((self.start[0] == 0 and self.lenB == self.end[1]) or
                 (self.start[1] == 0 and self.lenA == self.end[0])))

    def overlap(self):  # Overlap, ObjectStore.scala:119-135
        ahg = self.start[0] - self.start[1]
        bhg = self.lenB - self.lenA + ahg
        return ahg, bhg

    def overlap_valid(self, s):  # ObjectStore.scala:137-141
        ahg, bhg = self.overlap()
        return self.valid(s) and F32(abs(ahg)) < s.maxIgnore and F32(abs(bhg)) < s.maxIgnore

    def ovl_text(self):
        ahg, bhg = self.overlap()
        return "{OVL\nadj:N\nrds:%d,%d\nscr:0\nahg:%d\nbhg:%d\n}" % (self.idA, self.idB, ahg, bhg)


DUD = Alignment(0, 0, 0, 0, (0, 0), (0, 0), 0, 1)  # BioLibs.scala:22
DUD.alen = 0  # its alignA is "" although error == 1


# --------------------------------------------------------------------------
# BioLibs.scala
# --------------------------------------------------------------------------
def read_seq(text):  # BioLibs.readSeq :26-50 (java BufferedReader.readLine splitting)
    lines = text.replace("\r\n", "\n").replace("\r", "\n").split("\n")
    if text.endswith("\n") or text.endswith("\r"):
        lines = lines[:-1]
    if not lines or not lines[0].startswith(">"):
        raise ValueError("Invalid Sequence File")
    out, s = [], ""
    for line in lines[1:]:
        if line.startswith(">"):
            out.append(s.upper())
            s = ""
        else:
            s += line
    out.append(s.upper())
    return out  # ids are 1..len(out)


def generate_kmer_set(k, sid, seq):  # BioLibs.generateKmerSet :54-61
    d = F32(len(seq) - k)
    out = []
    for i in range(0, len(seq) - k + 1):
        with np.errstate(invalid="ignore", divide="ignore"):
            loc = F32(i) / d
        out.append(Kmer(sid, seq[i:i + k], loc))
    return out


def default_hoxd_table():  # BioLibs.defaultHOXD :119-140 (A0 C1 G2 T3)
    return [[91, -114, -31, -123], [-114, 100, -125, -31],
            [-31, -125, 100, -114], [-123, -31, -114, 91]]


_HX = {"A": 0, "C": 1, "G": 2, "T": 3}


class JvmError(Exception):
    """An exception that would end the reference run (NPE, MatchError, ...)."""


def _java_split(s):  # String.split(","): trailing empty strings removed
    if s == "":
        return [""]
    parts = s.split(",")
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def _java_trim(s):  # String.trim: code points <= U+0020 off both ends
    b, e = 0, len(s)
    while b < e and ord(s[b]) <= 0x20:
        b += 1
    while e > b and ord(s[e - 1]) <= 0x20:
        e -= 1
    return s[b:e]


def _java_parse_int(s):  # Integer.parseInt(s): [+-]?[0-9]+ within Int range
    t = s[1:] if s[:1] in ("+", "-") else s
    if not t or any(c not in "0123456789" for c in t):
        raise JvmError("NumberFormatException: " + repr(s))
    v = int(s)
    if not -2 ** 31 <= v < 2 ** 31:
        raise JvmError("NumberFormatException: " + repr(s))
    return v


def _java_read_lines(data):  # BufferedReader.readLine over the whole file
    out, cur, i = [], [], 0
    pending = False
    while i < len(data):
        c = data[i]
        if c in "\r\n":
            out.append("".join(cur))
            cur, pending = [], False
            if c == "\r" and i + 1 < len(data) and data[i + 1] == "\n":
                i += 1
        else:
            cur.append(c)
            pending = True
        i += 1
    if pending:
        out.append("".join(cur))
    return out


def read_hoxd(path):  # BioLibs.readHOXD :66-114 -> 4x4 table (A0 C1 G2 T3) or JvmError
    costs = [[0] * 4 for _ in range(4)]  # Array.ofDim(4,4) :68
    lines = _java_read_lines(open(path, "rb").read().decode("latin-1"))
    if len(lines) < 2:
        raise JvmError("NullPointerException: readLine() == null")
    col = _java_split(lines[1])  # :71
    li = 2
    while li < len(lines) and lines[li] != "":  # :75
        row = _java_split(lines[li])
        for i in range(1, len(row)):  # :77
            r0 = _java_trim(row[0])
            if not r0:
                raise JvmError("StringIndexOutOfBoundsException")
            if r0[0].upper() not in _HX:
                raise JvmError("MatchError")
            A = _HX[r0[0].upper()]
            if i >= len(col):
                raise JvmError("ArrayIndexOutOfBoundsException")
            ci = _java_trim(col[i])
            if not ci:
                raise JvmError("StringIndexOutOfBoundsException")
            if ci[0].upper() not in _HX:
                raise JvmError("MatchError")
            B = _HX[ci[0].upper()]
            costs[A][B] = _java_parse_int(row[i])  # :90
        li += 1
    return costs


def cost(s, a, b):  # the closure at :142-160 (MatchError on non-ACGT)
    return s.cost[_HX[a.upper()]][_HX[b.upper()]]


def fast_dovetail(idA, A, idB, B, s):  # BioLibs.generateFastDovetailAlignmentSet :596-822 (one B)
    gO, gE = s.gapOpen, s.gapExtend
    width = max(s.kmerSize, int(np.floor(F32(len(A)) * (F32(1) - s.minIdentity))) + 1)  # :619-620
    M = [[0] * (width + 1) for _ in range(len(A) + 1)]
    X = [[0] * (width + 1) for _ in range(len(A) + 1)]
    Y = [[0] * (width + 1) for _ in range(len(A) + 1)]
    for i in range(len(A)):  # :629-633
        M[i][0] = 0; X[i][0] = 0; Y[i][0] = gO + i * gE
    for i in range(width):  # :635-639
        M[0][i] = 0; X[0][i] = gO + i * gE; Y[0][i] = 0
    mx, maxLoc = 0, (0, 0)
    for i in range(1, len(A) + 1):  # :645-668
        for j in range(1, width + 1):
            M[i][j] = cost(s, A[i - 1], B[j - 1]) + max(max(M[i - 1][j - 1], Y[i - 1][j - 1]), max(X[i - 1][j - 1], 0))
            X[i][j] = gE + max(max(M[i][j - 1] + gO, Y[i][j - 1] + gO), max(X[i][j - 1], 0))
            Y[i][j] = gE + max(max(M[i - 1][j] + gO, Y[i - 1][j]), max(X[i - 1][j] + gO, 0))
            t = max(M[i][j], max(X[i][j], Y[i][j]))
            if t > mx:
                mx, maxLoc = t, (i, j)
    i, j = maxLoc  # :673-689
    mx = max(M[i][j], X[i][j], Y[i][j])
    while True:
        if i < 0 or j < 0:
            raise IndexError("degenerate phase-1 backtrack")
        if M[i][j] == mx:
            i -= 1; j -= 1
        elif X[i][j] == mx:
            j -= 1
        elif Y[i][j] == mx:
            i -= 1
        if i < 0 or j < 0:
            raise IndexError("degenerate phase-1 backtrack")
        mx = max(M[i][j], X[i][j], Y[i][j])
        if not mx > 0:
            break
    if j != 0:  # :694-695
        return DUD
    doveStart = i  # :703-705
    doveLength = len(A) - doveStart
    zeroRow = width // 2
    mx, maxLoc = 0, (0, 0)
    for u in range(0, doveLength + 1):  # :725-764
        for k in range(0, width + 1):
            i = u + doveStart
            j = k - zeroRow + u
            if i <= doveStart or j <= 0 or j > len(B):
                M[u][k] = 0; X[u][k] = 0; Y[u][k] = 0
            else:
                M[u][k] = (cost(s, A[i - 1], B[j - 1]) + max(max(M[u - 1][k], Y[u - 1][k]), max(X[u - 1][k], 0))) if u != 0 else 0
                X[u][k] = (gE + max(max(M[u][k - 1] + gO, Y[u][k - 1] + gO), max(X[u][k - 1], 0))) if k != 0 else 0
                if u != 0 and k != width:
                    Y[u][k] = gE + max(max(M[u - 1][k + 1] + gO, Y[u - 1][k + 1]), max(X[u - 1][k + 1] + gO, 0))
                else:
                    Y[u][k] = 0
            t = max(M[u][k], max(X[u][k], Y[u][k]))
            if t > mx:
                mx, maxLoc = t, (u, k)
    opt = maxLoc  # :768-809
    u, k = maxLoc
    c = e = 0
    mx = max(M[u][k], X[u][k], Y[u][k])
    while True:
        i = u + doveStart
        j = k - zeroRow + u
        if M[u][k] == mx:
            pa, pb = A[i - 1], B[j - 1]; u -= 1
        elif X[u][k] == mx:
            pa, pb = A[i - 1], "-"; k -= 1
        elif Y[u][k] == mx:
            pa, pb = "-", B[j - 1]; u -= 1; k += 1
        if pa != pb:
            e += 1
        else:
            c += 1
        mx = max(M[u][k], X[u][k], Y[u][k])
        if not mx > 0:
            break
    i = u + doveStart  # :812-819
    j = k - zeroRow + u
    newEnd = (opt[0] + doveStart, opt[1] - zeroRow + opt[0])
    return Alignment(len(A), len(B), idA, idB, (i, j), newEnd, c, e)


def local_alignment_set(maxL, idA, A, Bs, s):  # BioLibs.generateLocalAlignmentSet :267-368
    gO, gE = s.gapOpen, s.gapExtend
    M = [[0] * (maxL + 1) for _ in range(len(A) + 1)]  # :276-278, reused across the block
    X = [[0] * (maxL + 1) for _ in range(len(A) + 1)]
    Y = [[0] * (maxL + 1) for _ in range(len(A) + 1)]
    for i in range(len(A)):  # :281-285
        M[i][0] = 0; X[i][0] = 0; Y[i][0] = gO + i * gE
    for i in range(maxL):  # :287-291
        M[0][i] = 0; X[0][i] = gO + i * gE; Y[0][i] = 0
    out = []
    for idB, B in Bs:  # :293
        mx, maxLoc = 0, (0, 0)
        for i in range(1, len(A) + 1):  # :301-324
            for j in range(1, len(B) + 1):
                M[i][j] = cost(s, A[i - 1], B[j - 1]) + max(max(M[i - 1][j - 1], Y[i - 1][j - 1]),
                                                            max(X[i - 1][j - 1], 0))
                X[i][j] = gE + max(max(M[i][j - 1] + gO, Y[i][j - 1] + gO), max(X[i][j - 1], 0))
                Y[i][j] = gE + max(max(M[i - 1][j] + gO, Y[i - 1][j]), max(X[i - 1][j] + gO, 0))
                t = max(M[i][j], max(X[i][j], Y[i][j]))
                if t > mx:
                    mx, maxLoc = t, (i, j)
        opt = maxLoc  # :326-362
        i, j = maxLoc
        c = e = 0
        mx = max(M[i][j], X[i][j], Y[i][j])
        while True:
            if M[i][j] == mx:
                if i - 1 < 0 or j - 1 < 0:
                    raise IndexError("StringIndexOutOfBounds: degenerate local backtrack")
                pa, pb = A[i - 1], B[j - 1]; i -= 1; j -= 1
            elif X[i][j] == mx:
                pa, pb = A[i - 1], "-"; j -= 1
            elif Y[i][j] == mx:
                pa, pb = "-", B[j - 1]; i -= 1
            if pa != pb:
                e += 1
            else:
                c += 1
            mx = max(M[i][j], X[i][j], Y[i][j])
            if not mx > 0:
                break
        out.append(Alignment(len(A), len(B), idA, idB, (i, j), opt, c, e))  # :364
    return out


# --------------------------------------------------------------------------
# KmerTable.scala
# --------------------------------------------------------------------------
class KmerTable:
    def __init__(self):
        self.KmerData = TroveIntMap()
        self.PairData = TroveIntMap()
        self.DispatchData = TroveIntMap()
        self.SequenceData = {}
        self.pair_first_order = []  # distinct PairData keys in first-insertion order (diagnostic)

    def add_kmer_set(self, sid, seq, kmers):  # :41-53
        self.SequenceData[sid] = seq
        for s in kmers:
            if not self.KmerData.contains(s.int):
                self.KmerData.put(s.int, [])
            self.KmerData.get(s.int).append(s)

    def add_kmer_pair(self, a, b):  # :57-80
        if a.id == b.id:
            return
        if a.loc > b.loc:
            fst, snd = a, b
        else:
            fst, snd = b, a
        key = i32(fst.id << 16) ^ snd.id
        key = i32(key)
        if not self.PairData.contains(key):
            self.PairData.put(key, 0)
            self.pair_first_order.append(key)
        self.PairData.put(key, self.PairData.get(key) + 1)

    def calc_pair_data(self, s):  # :85-149
        for _, arr in self.KmerData.items():
            st = [k for k in arr if k.loc <= s.kmerHeadEdge]
            md = [k for k in arr if s.kmerMidLeadEdge <= k.loc and k.loc <= s.kmerMidTailEdge]
            en = [k for k in arr if s.kmerTailEdge <= k.loc]
            for a in st:
                for b in md:
                    self.add_kmer_pair(a, b)
            for a in en:
                for b in md:
                    self.add_kmer_pair(a, b)

    def calc_dispatch_data(self, s):  # :155-187
        for key, count in self.PairData.items():
            a = key >> 16
            b = i32((key << 16) & 0xFFFFFFFF) >> 16
            if s.minCollisions <= count <= s.maxCollisions:
                if not self.DispatchData.contains(a):
                    self.DispatchData.put(a, [])
                self.DispatchData.get(a).append(b)

    def dispatch_blocks(self, s):  # :246-273
        self.calc_pair_data(s)
        self.calc_dispatch_data(s)
        for lead, trails in self.DispatchData.items():
            for j in trails:
                if j not in self.SequenceData or lead not in self.SequenceData:
                    raise KeyError("NullPointerException: id %d/%d" % (lead, j))
            if len(trails) >= 1:
                yield lead, trails


def run(text, s, quadratic=False):
    """Project4 calc-overlaps path (:56-60): returns (.ovl text, table, alignments).
    quadratic=True is `--quadratic-align` (fdAlign = false, Project4.scala:187-189):
    calcLocalAlignmentSet -> generateLocalAlignmentSet (:599-604)."""
    seqs = read_seq(text)
    table = KmerTable()
    for idx, seq in enumerate(seqs):  # genMTKmerTable :531-563 (joined in read order)
        sid = idx + 1
        table.add_kmer_set(sid, seq, generate_kmer_set(s.kmerSize, sid, seq))
    aligns = []
    for lead, trails in table.dispatch_blocks(s):  # genBlockMTAlign :725-790
        A = table.SequenceData[lead]
        if quadratic:
            maxL = max(len(table.SequenceData[j]) for j in trails)  # KmerTable.scala:259-264
            block = local_alignment_set(maxL, lead, A, [(j, table.SequenceData[j]) for j in trails], s)
        else:
            block = [fast_dovetail(lead, A, j, table.SequenceData[j], s) for j in trails]
        aligns.extend(a for a in block if a.valid(s))
    out = "".join(a.ovl_text() + "\n" for a in aligns if a.overlap_valid(s))  # calcOverlaps :795-825
    return out, table, aligns
