"""Seeded read-name blocks for the tok3 name tokeniser tests: the name
formats search_trie special-cases (tokenise_name3.c:606-644: Illumina
lane:tile:x:y, IonTorrent, ONT uuids, PacBio), generic names, duplicates,
leading zeros, '\\0' and '\\n' separators, a partial last line, and the
failure cases (a byte >= 0x80, a control byte, more than 128 tokens)."""
import random


def _illumina(rng, n, paired=False):
    out, tile, x = [], 1101, 1000
    for i in range(n):
        if rng.random() < 0.05:
            tile += 1
            x = 1000
        x += rng.randint(0, 300)
        y = rng.randint(1000, 40000)
        nm = f"@A00123:8:H3VKJDSXY:{1 + (i * 4) // n}:{tile}:{x}:{y}"
        if paired:
            nm += f" {1 + (i & 1)}:N:0:ACGTACGT+TTGACCAA"
        out.append(nm)
    return out


def _srr(rng, n):
    return [f"SRR{1238539}.{i + 1} {i + 1} length={rng.choice([100, 101, 150])}"
            for i in range(n)]


def _ion(rng, n):
    return [f"ZX{rng.choice('ABC')}{rng.choice('DE')}:{rng.randint(0, 99999):05d}:{rng.randint(0, 99999):05d}"
            for _ in range(n)]


def _ont(rng, n):
    hx = "0123456789abcdef"
    out = []
    for i in range(n):
        u = "".join(rng.choice(hx) for _ in range(32))
        u = f"{u[:8]}-{u[8:12]}-{u[12:16]}-{u[16:20]}-{u[20:]}"
        out.append(u + f" runid=8a4b{i % 3} read={i * 7} ch={rng.randint(1, 512)} "
                   "start_time=2020-01-01T00:00:00Z")
    return out


def _pacbio(rng, n):
    mov = "m130802_221257_00127_c100560082550000001823094812221334_s1_p0"
    out, zmw = [], 100
    for i in range(n):
        if rng.random() < 0.6:
            zmw += rng.randint(1, 40)
        s = rng.randint(0, 20000)
        out.append(f"{mov}/{zmw}/{s}_{s + rng.randint(50, 5000)}")
    return out


def _zeros(rng, n):
    out, v = [], 0
    for i in range(n):
        v += rng.choice([1, 1, 1, 2, 255, 300])
        w = rng.choice([6, 6, 6, 8])
        out.append(f"read_{v % 10**w:0{w}d}/{rng.choice([1, 2])}#{i:03d}")
    return out


def _mixed(rng, n):
    pool = _illumina(rng, 20) + _srr(rng, 10) + ["x", "", "a:b", "007", "0", "A1B2C3", "a.b.c"]
    out = []
    for _ in range(n):
        nm = rng.choice(pool)
        if rng.random() < 0.3 and out:
            nm = rng.choice(out)             # an exact duplicate
        out.append(nm)
    return out


def _dups(rng, n):
    base = _illumina(rng, max(1, n // 4))
    return [base[i // 4] for i in range(n)]


def block(names, sep="\n", tail=True):
    b = sep.join(names)
    return (b + sep if tail else b).encode()


def cases():
    """(case name, block bytes) pairs; blocks the reference codes."""
    rng = random.Random(1238539)
    out = [
        ("illumina_1k", block(_illumina(rng, 1000))),
        ("illumina_paired_2k", block(_illumina(rng, 2000, paired=True))),
        ("illumina_nul_500", block(_illumina(rng, 500), sep="\0")),
        ("srr_3k", block(_srr(rng, 3000))),
        ("ion_800", block(_ion(rng, 800))),
        ("ont_300", block(_ont(rng, 300))),
        ("pacbio_600", block(_pacbio(rng, 600))),
        ("zeros_1k", block(_zeros(rng, 1000))),
        ("mixed_700", block(_mixed(rng, 700))),
        ("dups_400", block(_dups(rng, 400))),
        ("one_name", b"@read1\n"),
        ("one_empty", b"\n"),
        ("empties", b"\n\n\n\n"),
        ("partial_tail", block(_illumina(rng, 50), tail=False)),
        ("long_alpha", block(["A" * 200 + str(i) for i in range(30)])),
        ("tokens_127", block([".".join("a1" for _ in range(42)) + "x"] * 3)),
        ("illumina_20k", block(_illumina(rng, 20000, paired=True))),
    ]
    return out


def bad_cases():
    """Blocks the reference refuses (NULL)."""
    return [
        ("high_byte", b"@r1\n@r\xe92\n"),
        ("control_byte", b"@r1\n@r\x012\n"),
        ("tab_byte", b"@r1\tx\n"),
        ("tokens_200", block([".".join("a1" for _ in range(70))])),
        ("no_terminator", b"@read1"),
        ("empty", b""),
    ]
