"""Documents whose updates overlap the way snapshot + pending-log merges do: partial
overlaps (splices), same-clock blocks of different lengths, and Item-vs-GC ties at one
(client, clock) — the inconsistent arm of yrs' decoder comparator (update.rs:580-582) —
with decoder counts on both sides of Rust's 20-element insertion-sort threshold."""
import numpy as np


def _var(x):
    out = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _item(text):
    """String item, no origins, parent = root "t" (update.rs:433-488)."""
    t = text.encode()
    return bytes([0x04]) + _var(1) + _var(1) + b"t" + _var(len(t)) + t


def _gc(n):
    return bytes([0x00]) + _var(n)


def update(sections, ds=()):
    """sections: [(client, clock, [("i", text) | ("g", len)])]; ds: [(client, [(start, len)])]."""
    b = bytearray(_var(len(sections)))
    for c, k, blocks in sections:
        b += _var(len(blocks)) + _var(c) + _var(k)
        for kind, x in blocks:
            b += _item(x) if kind == "i" else _gc(x)
    b += _var(len(ds))
    for c, rs in ds:
        b += _var(c) + _var(len(rs))
        for s, n in rs:
            b += _var(s) + _var(n)
    return bytes(b)


def overlap_doc(rng, n_updates, n_clients=2, width=120, grid=4, gc_frac=0.4, snapshot=True):
    clients = [int(x) for x in rng.choice(2 ** 31, n_clients, replace=False)]
    ups = []
    if snapshot:  # one long section per client, Items and GCs, like a compacted document
        secs = []
        for c in clients:
            blocks, k = [], 0
            while k < width:
                n = int(rng.integers(3, 17))
                blocks.append(("g", n) if rng.random() < gc_frac else ("i", "".join(
                    chr(97 + int(v)) for v in rng.integers(0, 26, n))))
                k += n
            secs.append((c, 0, blocks))
        ups.append(update(secs))
    for _ in range(n_updates):
        if rng.random() < 0.1:
            c = clients[int(rng.integers(0, n_clients))]
            ups.append(update([], [(c, [(int(rng.integers(0, width)), int(rng.integers(1, 6)))])]))
            continue
        secs = []
        for c in rng.permutation(clients)[: int(rng.integers(1, min(2, n_clients) + 1))]:
            k0 = int(rng.integers(0, width // grid)) * grid  # starts on a grid: many same-clock ties
            blocks = []
            for _ in range(int(rng.integers(1, 4))):
                n = int(rng.integers(1, 9))
                blocks.append(("g", n) if rng.random() < gc_frac else ("i", "".join(
                    chr(97 + int(v)) for v in rng.integers(0, 26, n))))
            secs.append((int(c), k0, blocks))
        ups.append(update(secs))
    order = rng.permutation(len(ups))
    return [ups[i] for i in order]


def overlap_docs(seed, sizes=(2, 5, 12, 19, 20, 21, 22, 30, 60, 150)):
    rng = np.random.default_rng(seed)
    docs = []
    for n in sizes:
        for rep in range(4):
            docs.append(overlap_doc(rng, n, n_clients=1 + rep % 3, snapshot=rep != 3,
                                    gc_frac=(0.0, 0.4, 0.5, 1.0)[rep]))
    return docs
