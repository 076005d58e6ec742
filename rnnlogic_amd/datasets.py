"""Dataset access for the benchmark / parity workloads.

UMLS and kinship ship in the repo in the reference's own on-disk format
(data/<name>/{entities,relations}.dict, {train,valid,test}.txt; reference
src/data.py:18-99 reads exactly these files).  Their rule files
(data/<name>/mined_rules.txt) were mined by the reference miner
(miner/main.cpp, `-threads 1`, H column dropped).

FB15k-237 and WN18RR: the reference mount lacks train.txt
(/root/reference/.MISSING_LARGE_BLOBS), so the split files are packed as ids in
data/<name>.npz (tools/pack_datasets.py) and a seeded synthetic train graph is
generated here (SURVEY.md §8d recipe).  `materialize()` writes a directory in
the reference's format so that `KnowledgeGraph(path)` — ours and the
reference's — reads identical inputs.
"""
import hashlib
import json
import os

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")
# generated datasets (synthetic train graphs, RotatE tables) live outside the repo
BUILD = os.environ.get("RNNL_DATA_BUILD", "/tmp/rnnlogic_amd_data")

# Forward-triple counts of the real train splits (inverses are added on top).
PACKED = {
    "FB15k-237": dict(npz="fb15k237.npz", n_forward=272115, rotate_dim=1000, rotate_gamma=9.0,
                      sha256="bbe41f4a41d09309ca48ca0a3b971289c346215f8e0b2a2d5405962adeaec62c"),
    "wn18rr": dict(npz="wn18rr.npz", n_forward=86835, rotate_dim=500, rotate_gamma=6.0,
                   sha256="ade9fcb41fe32293d6b960968633b99b3c1196e45a703e51b1af33e285554e07"),
}
SHIPPED = ("umls", "kinship")


def synthesize_train(n_entities, n_relations, valid, test, n_forward, seed=0):
    """Seeded synthetic train graph with the real graph's marginals.

    Relations r < n_relations/2 are forward, r + n_relations/2 their inverses
    (as in the reference's relations.dict for both graphs).  Forward triples are
    drawn with relation frequency ~ valid+test counts (+0.5), heads/tails ~
    valid+test head/tail frequencies (+0.2); self-loops, duplicates and
    valid/test triples are rejected; every forward (h, r, t) is followed by its
    inverse (t, r + R/2, h).  Returns (2*n_forward, 3) int64 in file order.
    """
    half = n_relations // 2
    vt = np.concatenate([valid, test]).astype(np.int64)
    fwd = vt[vt[:, 1] < half]
    rel_p = np.bincount(fwd[:, 1], minlength=half).astype(np.float64) + 0.5
    head_p = np.bincount(fwd[:, 0], minlength=n_entities).astype(np.float64) + 0.2
    tail_p = np.bincount(fwd[:, 2], minlength=n_entities).astype(np.float64) + 0.2
    rel_p /= rel_p.sum()
    head_p /= head_p.sum()
    tail_p /= tail_p.sum()

    def key(h, r, t):
        return (r * n_entities + h) * n_entities + t

    forbidden = set(key(fwd[:, 0], fwd[:, 1], fwd[:, 2]).tolist())
    rng = np.random.RandomState(seed)
    chosen = []
    seen = set()
    need = n_forward
    while need > 0:
        m = int(need * 1.3) + 1024
        r = rng.choice(half, size=m, p=rel_p)
        h = rng.choice(n_entities, size=m, p=head_p)
        t = rng.choice(n_entities, size=m, p=tail_p)
        ok = h != t
        for hh, rr, tt in zip(h[ok].tolist(), r[ok].tolist(), t[ok].tolist()):
            k = (rr * n_entities + hh) * n_entities + tt
            if k in seen or k in forbidden:
                continue
            seen.add(k)
            chosen.append((hh, rr, tt))
            need -= 1
            if need == 0:
                break
    f = np.asarray(chosen, dtype=np.int64)
    inv = np.stack([f[:, 2], f[:, 1] + half, f[:, 0]], axis=1)
    out = np.empty((2 * len(f), 3), dtype=np.int64)
    out[0::2] = f
    out[1::2] = inv
    return out


def synthesize_rotate(n_entities, n_relations_fwd, dim, gamma, seed=0):
    """Seeded RotatE tables in the layout the reference loads
    (src/embedding.py:7-26): entity (|E|, 2D), relation (nrel_fwd, D), both
    U(-range, range) with range = (gamma + 2) / D (RotatE's embedding_range)."""
    rng = np.random.RandomState(seed + 1)
    rg = (gamma + 2.0) / dim
    eemb = rng.uniform(-rg, rg, size=(n_entities, 2 * dim)).astype(np.float32)
    remb = rng.uniform(-rg, rg, size=(n_relations_fwd, dim)).astype(np.float32)
    return eemb, remb


def _write_triples(path, trip):
    with open(path, "w") as f:
        f.write("".join("e%d\tr%d\te%d\n" % (h, r, t) for h, r, t in trip.tolist()))


def _sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def materialize(name, root=None, with_rotate=False):
    """Return a directory in the reference's format for dataset `name`.

    Shipped datasets return their in-repo directory.  Packed ones are written
    once under $RNNL_DATA_BUILD/<name>/ (default /tmp/rnnlogic_amd_data; names
    are synthetic: e<id>, r<id>).
    """
    if name in SHIPPED:
        return os.path.join(ROOT, name)
    if name not in PACKED:
        raise KeyError(name)
    spec = PACKED[name]
    out = os.path.join(root or BUILD, name)
    if not os.path.exists(os.path.join(out, "manifest.json")):
        # build in a private directory, then rename: concurrent ranks never see a partial dataset
        tmp = "%s.tmp.%d" % (out, os.getpid())
        os.makedirs(tmp, exist_ok=True)
        z = np.load(os.path.join(ROOT, spec["npz"]), allow_pickle=False)
        n_e, n_r = int(z["n_entities"]), int(z["n_relations"])
        with open(os.path.join(tmp, "entities.dict"), "w") as f:
            f.write("".join("%d\te%d\n" % (i, i) for i in range(n_e)))
        with open(os.path.join(tmp, "relations.dict"), "w") as f:
            f.write("".join("%d\tr%d\n" % (i, i) for i in range(n_r)))
        train = synthesize_train(n_e, n_r, z["valid"], z["test"], spec["n_forward"])
        _write_triples(os.path.join(tmp, "train.txt"), train)
        _write_triples(os.path.join(tmp, "valid.txt"), z["valid"])
        _write_triples(os.path.join(tmp, "test.txt"), z["test"])
        flat, ptr = z["rules_flat"], z["rules_ptr"]
        with open(os.path.join(tmp, "rnnlogic_rules.txt"), "w") as f:
            f.write("".join(" ".join(map(str, flat[ptr[i]:ptr[i + 1]].tolist())) + "\n"
                            for i in range(len(ptr) - 1)))
        digest = _sha256(os.path.join(tmp, "train.txt"))
        if digest != spec["sha256"]:
            raise RuntimeError("synthetic %s train graph differs from the one the golden fixtures were made "
                               "with (sha256 %s != %s)" % (name, digest, spec["sha256"]))
        with open(os.path.join(tmp, "manifest.json"), "w") as f:
            json.dump({"train_sha256": digest, "n_train": int(len(train)), "seed": 0}, f)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        try:
            os.rename(tmp, out)
        except OSError:  # another process won the race
            import shutil
            shutil.rmtree(tmp, ignore_errors=True)
    if with_rotate:
        rdir = os.path.join(out, "RotatE_%d" % spec["rotate_dim"])
        if not os.path.exists(os.path.join(rdir, "config.json")):
            tmp = "%s.tmp.%d" % (rdir, os.getpid())
            os.makedirs(tmp, exist_ok=True)
            z = np.load(os.path.join(ROOT, spec["npz"]), allow_pickle=False)
            n_e, n_r = int(z["n_entities"]), int(z["n_relations"])
            eemb, remb = synthesize_rotate(n_e, n_r // 2, spec["rotate_dim"], spec["rotate_gamma"])
            np.save(os.path.join(tmp, "entity_embedding.npy"), eemb)
            np.save(os.path.join(tmp, "relation_embedding.npy"), remb)
            with open(os.path.join(tmp, "config.json"), "w") as f:
                json.dump({"hidden_dim": spec["rotate_dim"], "gamma": spec["rotate_gamma"],
                           "nentity": n_e, "nrelation": n_r // 2, "synthetic": True}, f)
            try:
                os.rename(tmp, rdir)
            except OSError:
                import shutil
                shutil.rmtree(tmp, ignore_errors=True)
    return out


def rule_file(name):
    """Path of the rule file used for dataset `name`."""
    if name in SHIPPED:
        return os.path.join(ROOT, name, "mined_rules.txt")
    return os.path.join(materialize(name), "rnnlogic_rules.txt")


def rotate_path(name, dim=None):
    if name in SHIPPED:
        return os.path.join(ROOT, name, "RotatE_%d" % (dim or (200 if name == "umls" else 1000)))
    return os.path.join(materialize(name, with_rotate=True), "RotatE_%d" % PACKED[name]["rotate_dim"])
