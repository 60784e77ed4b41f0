"""Damaged and hostile BAM / BGZF inputs to the host decoder (csrc/bcio.cpp): every one must end
in a format error, never in a read past the mapped file or an oversized allocation.  The reference
leaves this to htslib through pysam (main.py:119-127); its only guard of its own is the `.at()`
of count.cpp:60-65,85.  These inputs are also what `make -C basecount_amd/csrc asan` runs under
AddressSanitizer/UBSan (scripts/asan.sh)."""
import struct
import zlib

import pytest

from basecount_amd import synth
from basecount_amd.bam import BamFile


def _deflate(raw: bytes) -> bytes:
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    return c.compress(raw) + c.flush()


def bgzf_block(raw: bytes, *, bsize=None, xlen=None, extra=None, isize=None) -> bytes:
    """One BGZF block (RFC 1952 member with the BC extra subfield), fields overridable."""
    cdata = _deflate(raw)
    if extra is None:
        extra = b"BC" + struct.pack("<H", 2) + struct.pack("<H", 0)  # BSIZE patched below
    xl = len(extra) if xlen is None else xlen
    total = 12 + len(extra) + len(cdata) + 8
    bs = total - 1 if bsize is None else bsize
    if extra[:2] == b"BC" and len(extra) >= 6:
        extra = extra[:4] + struct.pack("<H", bs & 0xFFFF) + extra[6:]
    head = bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255]) + struct.pack("<H", xl)
    tail = struct.pack("<II", zlib.crc32(raw), len(raw) if isize is None else isize)
    return head + extra + cdata + tail


EOF_BLOCK = bgzf_block(b"")


def bam_header(refs=(("chrA", 1000),)) -> bytes:
    text = b"@HD\tVN:1.6\n"
    out = b"BAM\1" + struct.pack("<i", len(text)) + text + struct.pack("<i", len(refs))
    for name, ln in refs:
        nm = name.encode() + b"\0"
        out += struct.pack("<i", len(nm)) + nm + struct.pack("<i", ln)
    return out


def bam_record(*, tid=0, pos=10, mapq=60, flag=0, cigar=((0, 4),), seq=b"ACGT", qual=None,
               l_seq=None, n_cigar=None, l_read_name=None, block_size=None) -> bytes:
    name = b"r\0"
    codes = {c: i for i, c in enumerate(b"=ACMGRSVTWYHKDBN")}
    packed = bytearray((len(seq) + 1) // 2)
    for i, ch in enumerate(seq):
        packed[i // 2] |= codes[ch] << (4 if i % 2 == 0 else 0)
    q = bytes([30] * len(seq)) if qual is None else qual
    cig = b"".join(struct.pack("<I", (ln << 4) | op) for op, ln in cigar)
    body = struct.pack("<iiBBHHHiiii", tid, pos,
                       len(name) if l_read_name is None else l_read_name, mapq, 4680,
                       len(cigar) if n_cigar is None else n_cigar, flag,
                       len(seq) if l_seq is None else l_seq, -1, -1, 0)
    body += name + cig + bytes(packed) + q
    return struct.pack("<I", len(body) if block_size is None else block_size) + body


def write(tmp_path, blob: bytes, name="x.bam") -> str:
    p = tmp_path / name
    p.write_bytes(blob)
    return str(p)


def test_crafted_valid_file_decodes(tmp_path):
    """The crafting helpers themselves produce a file the decoder accepts (control case)."""
    raw = bam_header() + bam_record() + bam_record(pos=20, seq=b"ACGTN", cigar=((4, 1), (0, 4)))
    p = write(tmp_path, bgzf_block(raw) + EOF_BLOCK)
    with BamFile(p) as f:
        assert f.n_records == 2
        assert list(f.pos) == [10, 20]
        assert list(f.qstart) == [0, 1]


BAD_BLOCKS = {
    # BSIZE smaller than its own header: clen = bsize - xlen - 20 would underflow
    "bsize_below_header": lambda raw: bgzf_block(raw, bsize=30),
    # XLEN running past the end of the file
    "xlen_past_file": lambda raw: (bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255]) + struct.pack("<H", 60000)
                                   + b"BC" + struct.pack("<HH", 2, 100)),
    # a subfield whose length runs past XLEN
    "subfield_past_xlen": lambda raw: bgzf_block(raw, extra=b"XY" + struct.pack("<H", 40) + b"\0\0"),
    # no BC subfield at all
    "no_bc_subfield": lambda raw: bgzf_block(raw, extra=b"XY" + struct.pack("<H", 2) + b"\0\0"),
    # ISIZE claims more than the 64 KiB a BGZF block may hold
    "isize_over_64k": lambda raw: bgzf_block(raw, isize=1 << 30),
    # ISIZE disagreeing with the deflate stream
    "isize_mismatch": lambda raw: bgzf_block(raw, isize=len(raw) + 3),
    # BSIZE past the end of the file
    "bsize_past_file": lambda raw: bgzf_block(raw, bsize=60000),
    # not gzip at all
    "bad_magic": lambda raw: b"\x1f\x8c" + bgzf_block(raw)[2:],
    # header cut short
    "short_header": lambda raw: bgzf_block(raw)[:14],
}


@pytest.mark.parametrize("case", sorted(BAD_BLOCKS))
def test_bad_bgzf_block(tmp_path, case):
    raw = bam_header() + bam_record()
    p = write(tmp_path, BAD_BLOCKS[case](raw))
    with pytest.raises(Exception) as ei:
        BamFile(p)
    assert "BGZF" in str(ei.value) or "inflate" in str(ei.value) or "gzip" in str(ei.value)


BAD_RECORDS = {
    # l_seq far larger than the record: would size the sequence arrays from a hostile value
    "l_seq_huge": dict(l_seq=0x7FFFFFFF),
    "l_seq_past_record": dict(l_seq=400),
    "l_seq_negative": dict(l_seq=-5),
    # n_cigar past the record (and the block)
    "n_cigar_past_record": dict(n_cigar=5000),
    # read name length (the low byte of bin_mq_nl) overflowing the record
    "read_name_overflow": dict(l_read_name=255),
    # block_size below the fixed 32-byte part
    "block_size_tiny": dict(block_size=8),
    # block_size past the end of the inflated data
    "block_size_past_data": dict(block_size=10_000),
}


@pytest.mark.parametrize("case", sorted(BAD_RECORDS))
def test_bad_bam_record(tmp_path, case):
    raw = bam_header() + bam_record() + bam_record(pos=50, **BAD_RECORDS[case])
    p = write(tmp_path, bgzf_block(raw) + EOF_BLOCK)
    with pytest.raises(Exception) as ei:
        BamFile(p)
    assert "BAM" in str(ei.value) or "record" in str(ei.value) or "l_seq" in str(ei.value)


@pytest.mark.parametrize("case", ["no_magic", "text_len_past_data", "n_ref_truncated", "name_len_zero"])
def test_bad_bam_header(tmp_path, case):
    h = bam_header()
    if case == "no_magic":
        h = b"BAX\1" + h[4:]
    elif case == "text_len_past_data":
        h = h[:4] + struct.pack("<i", 1 << 20) + h[8:]
    elif case == "n_ref_truncated":
        h = h[: len(h) - 6]
    else:
        h = h[: h.index(b"chrA") - 4] + struct.pack("<i", 0) + h[h.index(b"chrA"):]
    p = write(tmp_path, bgzf_block(h) + EOF_BLOCK)
    with pytest.raises(Exception):
        BamFile(p)


def test_truncated_file_every_cut(tmp_path):
    """A real multi-block BAM cut at many offsets: each cut either still decodes a prefix-free
    valid file (only at block boundaries) or fails cleanly."""
    rs = synth.make_reads([("chrA", 3_000)], 400, True, 9)
    full = write(tmp_path, b"", "full.bam")
    synth.write_bam(rs, full)
    data = open(full, "rb").read()
    for cut in list(range(1, 64)) + list(range(64, len(data), max(1, len(data) // 97))):
        p = write(tmp_path, data[:cut], "cut.bam")
        try:
            with BamFile(p) as f:
                assert f.n_records <= rs.n
        except Exception:
            pass
