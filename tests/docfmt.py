"""Test helpers for the binary document format (test-side only)."""
import hashlib
import zlib


def uleb(b, off):
    v = sh = 0
    while True:
        x = b[off]
        off += 1
        v |= (x & 0x7f) << sh
        sh += 7
        if not x & 0x80:
            return v, off


def put_uleb(v):
    out = bytearray()
    while True:
        x = v & 0x7f
        v >>= 7
        out.append(x | (0x80 if v else 0))
        if not v:
            return bytes(out)


def deflate_raw(data):
    c = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
    return c.compress(data) + c.flush()


def to_saved_form(chunk):
    """Uncompressed document chunk -> save() form: columns >= 256 bytes DEFLATE-compressed
    (columnar.js:1052-1057) and the checksum recomputed (columnar.js:659-686)."""
    assert chunk[:4] == b"\x85\x6f\x4a\x83" and chunk[8] == 0
    ln, off = uleb(chunk, 9)
    data = chunk[off:off + ln]
    p = 0
    na, p = uleb(data, p)
    for _ in range(na):
        l, p = uleb(data, p)
        p += l
    nh, p = uleb(data, p)
    p += 32 * nh
    pre = data[:p]
    tables = []
    for _ in range(2):
        nc, p = uleb(data, p)
        cols = []
        for _ in range(nc):
            cid, p = uleb(data, p)
            cl, p = uleb(data, p)
            cols.append([cid, cl])
        tables.append(cols)
    for cols in tables:
        for c in cols:
            c.append(data[p:p + c[1]])
            p += c[1]
    post = data[p:]
    changed = False
    for cols in tables:
        for c in cols:
            if len(c[2]) >= 256:
                c[2] = deflate_raw(c[2])
                c[0] |= 8
                changed = True
    if not changed:
        return chunk
    body = bytearray(pre)
    for cols in tables:
        body += put_uleb(len(cols))
        for c in cols:
            body += put_uleb(c[0]) + put_uleb(len(c[2]))
    for cols in tables:
        for c in cols:
            body += c[2]
    body += post
    hdr = b"\x00" + put_uleb(len(body))
    h = hashlib.sha256(hdr + bytes(body)).digest()
    return b"\x85\x6f\x4a\x83" + h[:4] + hdr + bytes(body)
