"""Test-side restatement of the compact StatusUpdate stream (include/avhip.h,
av_compact_header): encodes canonical packed update words the way
av_fetch_compact lays them out, so the CPU tests can check av_compact_expand
and the GPU tests can compare the device encoder's bytes exactly."""
import numpy as np

HEADER = np.dtype([("magic", "<u4"), ("version", "<u4"), ("log_base", "<i8"), ("n_updates", "<i8"),
                   ("bytes", "<i8"), ("node_base", "<i8"), ("target_base", "<i8"), ("n_rounds", "<i4"),
                   ("chunks", "<i4"), ("chunk_nodes", "<i4"), ("code_bytes", "<i4"), ("target_bits", "<i4"),
                   ("slot_bits", "<i4"), ("round_shift", "<i4"), ("reserved", "<i4")])
MAGIC, VERSION, CHUNK_NODES = 0x31435641, 1, 4096


def bits_for(n):
    b = 0
    while b < 32 and (1 << b) < n:
        b += 1
    return b


def encode(words, *, log_base, n_rounds, node_base, n_local, target_base, n_targets_local, k,
           chunk_nodes=CHUNK_NODES, round_shift=52):
    """Packed words (sorted canonical, round fields relative to log_base) -> stream bytes."""
    w = np.asarray(words, np.uint64)
    assert np.all(w[1:] >= w[:-1])
    tb, sb = bits_for(n_targets_local), bits_for(k)
    cw = 2 if sb + tb + 2 <= 16 else 4
    chunks = (n_local + chunk_nodes - 1) // chunk_nodes
    rr = (w >> np.uint64(round_shift)).astype(np.int64)
    node = ((w >> np.uint64(28)) & np.uint64((1 << (round_shift - 28)) - 1)).astype(np.int64)
    slot = ((w >> np.uint64(24)) & np.uint64(0xF)).astype(np.int64)
    tl = ((w >> np.uint64(2)) & np.uint64(0x3FFFFF)).astype(np.int64) - target_base
    st = (w & np.uint64(3)).astype(np.int64)
    assert np.all(rr < n_rounds) and np.all((node >= node_base) & (node < node_base + n_local))
    codes = (slot << (tb + 2)) | (tl << 2) | st
    key = rr * n_local + (node - node_base)
    # groups
    body = bytearray()
    idx = np.zeros((n_rounds * chunks + 1, 2), np.uint64)
    uniq, first = (np.unique(key, return_index=True) if key.size else (np.zeros(0, np.int64), np.zeros(0, np.int64)))
    bounds = list(first) + [key.size]
    gi = 0
    done = 0
    for r in range(n_rounds):
        for c in range(chunks):
            lo_key = r * n_local + c * chunk_nodes
            hi_key = r * n_local + min((c + 1) * chunk_nodes, n_local)
            idx[r * chunks + c] = (len(body), done)
            while gi < uniq.size and uniq[gi] < hi_key:
                assert uniq[gi] >= lo_key
                a, b = bounds[gi], bounds[gi + 1]
                n = b - a
                body += np.array([node[a], n], "<u4").tobytes()
                cb = codes[a:b].astype("<u2" if cw == 2 else "<u4").tobytes()
                body += cb + b"\0" * ((-len(cb)) % 4)
                done += n
                gi += 1
    idx[-1] = (len(body), done)
    h = np.zeros(1, HEADER)
    total = HEADER.itemsize + idx.nbytes + len(body)
    for name, v in (("magic", MAGIC), ("version", VERSION), ("log_base", log_base), ("n_updates", w.size),
                    ("bytes", total), ("node_base", node_base), ("target_base", target_base),
                    ("n_rounds", n_rounds), ("chunks", chunks), ("chunk_nodes", chunk_nodes), ("code_bytes", cw),
                    ("target_bits", tb), ("slot_bits", sb), ("round_shift", round_shift)):
        h[name] = v
    return np.frombuffer(h.tobytes() + idx.astype("<u8").tobytes() + bytes(body), np.uint8).copy()
