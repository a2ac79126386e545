"""Reader for the .fqz5 container as fqzcomp5 writes it, for the parity
tests (test infrastructure): header `FQZ5\\1\\1\\0\\0` + u64 index offset
(fqzcomp5.c:2563-2575), then blocks (encode_block, fqzcomp5.c:2147-2280):

    u32 block_size (bytes after this field)   u32 nrec   u32 crc32(bytes 12..)
    names    u32 u_len, u8 strat, u32 c_len, c_len bytes
    lengths  u8 nb > 0: varint fixed length | u8 0, u32 blen, blen bytes of varints
    seq      u8 strat, u32 u_len, u32 c_len, c_len bytes
    qual     u8 strat, u32 u_len, u32 c_len, c_len bytes

and the index at the header's offset (fqzcomp5.c:2606-2630)."""
import dataclasses
import struct
import zlib

MAGIC = b"FQZ5\x01\x01\x00\x00"


@dataclasses.dataclass
class Section:
    strat: int
    u_len: int
    data: bytes


@dataclasses.dataclass
class Block:
    nrec: int
    crc_ok: bool
    names: Section
    fixed_len: int          # 0 when the lengths are variable
    seq: Section
    qual: Section


def _sec(buf, p):
    strat = buf[p]
    u, c = struct.unpack_from("<II", buf, p + 1)
    return Section(strat, u, bytes(buf[p + 9:p + 9 + c])), p + 9 + c


def raw_blocks(path):
    """Each block's bytes as the file holds them (block_size field first)."""
    buf = open(path, "rb").read()
    (idx,) = struct.unpack_from("<Q", buf, 8)
    end = idx if idx else len(buf)
    p, out = 16, []
    while p < end:
        (bsz,) = struct.unpack_from("<I", buf, p)
        out.append(bytes(buf[p:p + 4 + bsz]))
        p += 4 + bsz
    return out


def read(path):
    buf = open(path, "rb").read()
    assert buf[:8] == MAGIC, buf[:8]
    (idx,) = struct.unpack_from("<Q", buf, 8)
    end = idx if idx else len(buf)
    p, blocks = 16, []
    while p < end:
        bsz, nrec, crc = struct.unpack_from("<III", buf, p)
        bend = p + 4 + bsz
        crc_ok = zlib.crc32(buf[p + 12:bend]) == crc
        q = p + 12
        u, strat, c = struct.unpack_from("<IBI", buf, q)
        names = Section(strat, u, bytes(buf[q + 9:q + 9 + c]))
        q += 9 + c
        nb = buf[q]
        fixed = 0
        if nb:
            v, s = 0, 0
            q += 1
            while True:                      # big-endian 7-bit varint (varint.h:206)
                b = buf[q]
                q += 1
                v = (v << 7) | (b & 0x7f)
                if not b & 0x80:
                    break
                s += 1
            fixed = v
        else:
            (blen,) = struct.unpack_from("<I", buf, q + 1)
            q += 5 + blen
        seq, q = _sec(buf, q)
        qual, q = _sec(buf, q)
        assert q == bend, (q, bend)
        blocks.append(Block(nrec, crc_ok, names, fixed, seq, qual))
        p = bend
    return blocks


MAGIC_V10 = b"FQZ5\x01\x00\x00\x00"     # fqzcomp5.c:155


def downgrade(buf: bytes, version: str) -> bytes:
    """A v1.1 container rewritten in an older layout the reference still
    decodes (read_header, fqzcomp5.c:2578-2603; decode_block :2300-2318):
    "v1.0": magic FQZ5\\1\\0\\0\\0, no CRC field in the blocks (block_size 4
    smaller), the index offsets moved to match; "old": no file header, no CRC
    fields and no index (the decoder reads blocks up to the end)."""
    assert buf[:8] == MAGIC and version in ("v1.0", "old")
    (idx,) = struct.unpack_from("<Q", buf, 8)
    end = idx if idx else len(buf)
    p, blocks = 16, []
    while p < end:
        (bsz,) = struct.unpack_from("<I", buf, p)
        blk = buf[p:p + 4 + bsz]
        blocks.append(struct.pack("<I", bsz - 4) + blk[4:8] + blk[12:])
        p += 4 + bsz
    if version == "old":
        return b"".join(blocks)
    out, offs, at = [], [], 16
    for b in blocks:
        offs.append(at)
        at += len(b)
    tail = b""
    if idx:
        (n,) = struct.unpack_from("<I", buf, idx + 8)
        assert n == len(blocks)
        ent = [struct.unpack_from("<QII", buf, idx + 12 + 16 * i) for i in range(n)]
        tail = buf[idx:idx + 12] + b"".join(struct.pack("<QII", o, u, r)
                                            for o, (_, u, r) in zip(offs, ent))
    return MAGIC_V10 + struct.pack("<Q", at if idx else 0) + b"".join(blocks) + tail
