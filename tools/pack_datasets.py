"""Pack the reference's FB15k-237 / WN18RR split files into compact id arrays.

Run once in the build container (it reads /root/reference/data, which does not
exist on the GPU box).  Output: data/<name>.npz with

    n_entities, n_relations          scalars
    valid, test                      (N, 3) int32 (h, r, t) in file order
    rules_flat, rules_ptr            rnnlogic_rules.txt as a CSR of int32 tokens
                                     (head, body...) in file order

Entity/relation *names* are not kept: every consumer on the hot path works on
ids (reference src/data.py:18-28 maps names to ids once).  The train split of
both graphs is absent from the reference mount (.MISSING_LARGE_BLOBS), so a
seeded synthetic train graph is generated on demand by
rnnlogic_amd.datasets.synthesize_train.
"""
import os
import sys

import numpy as np

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data")


def read_dict(path):
    m = {}
    with open(path) as f:
        for line in f:
            i, name = line.rstrip("\n").split("\t")
            m[name] = int(i)
    return m


def read_triples(path, e2i, r2i):
    out = []
    with open(path) as f:
        for line in f:
            h, r, t = line.rstrip("\n").split("\t")
            out.append((e2i[h], r2i[r], e2i[t]))
    return np.asarray(out, dtype=np.int32).reshape(-1, 3)


def read_rules(path):
    flat, ptr = [], [0]
    with open(path) as f:
        for line in f:
            toks = [int(x) for x in line.split()]
            flat.extend(toks)
            ptr.append(len(flat))
    return np.asarray(flat, dtype=np.int32), np.asarray(ptr, dtype=np.int64)


def pack(name, out_name):
    d = os.path.join(REF, name)
    e2i = read_dict(os.path.join(d, "entities.dict"))
    r2i = read_dict(os.path.join(d, "relations.dict"))
    valid = read_triples(os.path.join(d, "valid.txt"), e2i, r2i)
    test = read_triples(os.path.join(d, "test.txt"), e2i, r2i)
    flat, ptr = read_rules(os.path.join(d, "rnnlogic_rules.txt"))
    path = os.path.join(OUT, out_name + ".npz")
    np.savez_compressed(path, n_entities=np.int64(len(e2i)), n_relations=np.int64(len(r2i)),
                        valid=valid, test=test, rules_flat=flat, rules_ptr=ptr)
    print(path, len(e2i), len(r2i), valid.shape, test.shape, len(ptr) - 1)


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference data not mounted")
    pack("FB15k-237", "fb15k237")
    pack("wn18rr", "wn18rr")
