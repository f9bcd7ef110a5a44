"""Test-only writer of LMDB data files (data version 1, 64-bit layout) used
to exercise the native read-only reader (csrc/runtime/lmdb_reader.cc): meta
pages 0/1 (the newer txnid wins), leaf pages, a branch level when the keys
do not fit one leaf, and overflow pages for values too large for a leaf.
Neither liblmdb nor the lmdb module exists in this environment and the
reference ships no LMDB file, so the layout follows LMDB's documented
on-disk structures (parity with real liblmdb output is unpinned)."""
import os
import struct

P_BRANCH, P_LEAF, P_OVERFLOW, P_META = 0x01, 0x02, 0x04, 0x08
F_BIGDATA = 0x01
P_INVALID = 0xFFFFFFFFFFFFFFFF


def _node(key: bytes, data: bytes, big_pg=None) -> bytes:
    if big_pg is not None:
        dsz = len(data)
        body = key + struct.pack("<Q", big_pg)
        flags = F_BIGDATA
    else:
        dsz = len(data)
        body = key + data
        flags = 0
    n = struct.pack("<HHHH", dsz & 0xFFFF, dsz >> 16, flags, len(key)) + body
    return n + (b"\0" if len(n) % 2 else b"")


def _branch_node(key: bytes, child: int) -> bytes:
    n = struct.pack("<HHHH", child & 0xFFFF, (child >> 16) & 0xFFFF, (child >> 32) & 0xFFFF, len(key)) + key
    return n + (b"\0" if len(n) % 2 else b"")


def _page(pgno: int, flags: int, nodes, psize: int) -> bytearray:
    p = bytearray(psize)
    upper = psize
    ptrs = []
    for n in nodes:
        upper -= len(n)
        p[upper:upper + len(n)] = n
        ptrs.append(upper)
    lower = 16 + 2 * len(ptrs)
    assert lower <= upper, "page overflow"
    struct.pack_into("<QHHHH", p, 0, pgno, 0, flags, lower, upper)
    for i, o in enumerate(ptrs):
        struct.pack_into("<H", p, 16 + 2 * i, o)
    return p


def write_lmdb(path: str, items, psize: int = 4096, leaf_limit: int = 0) -> None:
    """items: (key bytes, value bytes) pairs; keys are written sorted."""
    items = sorted(items)
    os.makedirs(path, exist_ok=True)
    pages = {}
    nxt = [2]

    def alloc(n=1):
        pg = nxt[0]
        nxt[0] += n
        return pg

    big_limit = psize // 4
    leaves, cur, used = [], [], 16
    ovf = 0
    for k, v in items:
        if len(v) > big_limit:
            npg = (16 + len(v) + psize - 1) // psize
            opg = alloc(npg)
            buf = bytearray(npg * psize)
            struct.pack_into("<QHHI", buf, 0, opg, 0, P_OVERFLOW, npg)
            buf[16:16 + len(v)] = v
            for i in range(npg):
                pages[opg + i] = buf[i * psize:(i + 1) * psize]
            node = _node(k, v, big_pg=opg)
            ovf += npg
        else:
            node = _node(k, v)
        if cur and (used + 2 + len(node) > psize or (leaf_limit and len(cur) >= leaf_limit)):
            leaves.append(cur)
            cur, used = [], 16
        cur.append((k, node))
        used += 2 + len(node)
    if cur:
        leaves.append(cur)
    leaf_pgs = []
    for lf in leaves:
        pg = alloc()
        pages[pg] = _page(pg, P_LEAF, [n for _, n in lf], psize)
        leaf_pgs.append((lf[0][0], pg))
    depth, nbranch = 1, 0
    level = leaf_pgs
    while len(level) > 1:
        depth += 1
        nxt_level = []
        for i in range(0, len(level), 64):
            grp = level[i:i + 64]
            pg = alloc()
            nodes = [_branch_node(b"" if j == 0 else k, c) for j, (k, c) in enumerate(grp)]
            pages[pg] = _page(pg, P_BRANCH, nodes, psize)
            nbranch += 1
            nxt_level.append((grp[0][0], pg))
        level = nxt_level
    root = level[0][1] if level else P_INVALID

    def meta(pgno: int, txnid: int, root_pg: int) -> bytearray:
        p = bytearray(psize)
        struct.pack_into("<QHHHH", p, 0, pgno, 0, P_META, 0, 0)
        struct.pack_into("<IIQQ", p, 16, 0xBEEFC0DE, 1, 0, nxt[0] * psize)
        free_db = struct.pack("<IHHQQQQQ", psize, 0, 0, 0, 0, 0, 0, P_INVALID)
        main_db = struct.pack("<IHHQQQQQ", 0, 0, depth if items else 0, nbranch, len(leaf_pgs), ovf, len(items),
                              root_pg)
        p[40:88] = free_db
        p[88:136] = main_db
        struct.pack_into("<QQ", p, 136, nxt[0] - 1, txnid)
        return p

    pages[0] = meta(0, 1, P_INVALID)   # stale meta (older txn, empty db)
    pages[1] = meta(1, 2, root)        # current meta
    with open(os.path.join(path, "data.mdb"), "wb") as f:
        for pg in range(nxt[0]):
            f.write(bytes(pages.get(pg, bytearray(psize))))


def datum(channels: int, height: int, width: int, pixels: bytes, label: int) -> bytes:
    """Caffe Datum protobuf encoding (channels=1 height=2 width=3 data=4 label=5)."""
    def varint(v):
        out = bytearray()
        while True:
            b = v & 0x7F
            v >>= 7
            out.append(b | (0x80 if v else 0))
            if not v:
                return bytes(out)
    return (b"\x08" + varint(channels) + b"\x10" + varint(height) + b"\x18" + varint(width) +
            b"\x22" + varint(len(pixels)) + pixels + b"\x28" + varint(label))
