"""TEST INFRASTRUCTURE ONLY (never shipped, never measured).

Restatement of the reference verkle tree (/root/reference/verkle-tree/src): `Node`
(node.rs:35-49) with `insert` (node.rs:133-204), `get_stem` / `get_value` (node.rs:74-131),
`path_to_stem` (node.rs:97-120) and the recursive `gen_commitment` (node.rs:205-277), and the
`VerkleTree` wrappers `insert_single` / `get_single` / `commitment` (lib.rs:112-129), for
keys of N u8 units and U256 values split into (low 16 bytes, high 16 bytes) LE Fr halves
(the reference tests' SplittableValue, lib.rs:186-194). The reference's quirks are kept:
the stem is the whole key (lib.rs:61-67), extension commits have width N (node.rs:226-239),
internal commits width 256 (node.rs:264), splits key the new internal node by the first
differing unit even when that skips levels (node.rs:176-185), and inserting a key that
reaches an extension with another stem raises (the reference panics, node.rs:148-150).

`commit(values)` is supplied by the caller: inner_product of the first len(values) CRS
points with the values (utils.rs:16-19 via IPA/KZG::commit), giving a point or None.
"""
from .arkser import to_data_item
from .curves import BN254

R = BN254.r


class VerklePanic(Exception):
    """the reference panics (node.rs:148-150, or an out-of-bounds stem index)"""


class Node:
    def __init__(self, ext, stem=None, leaves=None, children=None):
        self.ext = ext
        self.stem = stem
        self.leaves = leaves if leaves is not None else {}
        self.children = children if children is not None else {}
        self.commit = None
        self.has_commit = False


def _split(value):
    return int.from_bytes(value[:16], "little") % R, int.from_bytes(value[16:32], "little") % R


def _next_diff_depth(a, b, cur, N):  # lib.rs:49-58
    d = cur + 1
    while d < N and a[d] == b[d]:
        d += 1
    return d


class VerkleTree:
    def __init__(self, N):
        self.N = N
        self.root = Node(False)

    # node.rs:133-204
    def _insert(self, node, stem, values, cur_depth):
        N = self.N
        if node.ext:
            if node.stem != stem:
                raise VerklePanic("Traversed to extension node with differing stem")
            node.has_commit = False
            for k, v in values:
                node.leaves[k] = v
            return
        node.has_commit = False
        k = stem[cur_depth]
        child = node.children.get(k)
        if child is None:
            node.children[k] = Node(True, stem, dict(values))
            return
        if child.ext:
            if stem == child.stem or cur_depth == N - 2:
                self._insert(child, stem, values, cur_depth + 1)
            else:
                depth = _next_diff_depth(child.stem, stem, cur_depth, N)
                if depth >= N:
                    raise VerklePanic("index out of bounds")
                node.children[k] = Node(False, children={stem[depth]: Node(True, stem, dict(values)),
                                                          child.stem[depth]: child})
        else:
            self._insert(child, stem, values, cur_depth + 1)

    def _check_insert(self, stem):
        """the reference clears commitments on the way down before it panics; a panicking
        insert is rejected here before any change (the engine does the same)"""
        node, d, N = self.root, 0, self.N
        while True:
            if node.ext:
                if node.stem != stem:
                    raise VerklePanic("Traversed to extension node with differing stem")
                return
            child = node.children.get(stem[d])
            if child is None:
                return
            if child.ext and not (stem == child.stem or d == N - 2):
                if _next_diff_depth(child.stem, stem, d, N) >= N:
                    raise VerklePanic("index out of bounds")
                return
            node, d = child, d + 1

    def insert_single(self, key, value):  # lib.rs:112-116
        stem = tuple(key)
        self._check_insert(stem)
        self._insert(self.root, stem, [(key[-1], bytes(value))], 0)

    def _get_stem(self, node, stem, cur_depth):  # node.rs:74-95
        if node.ext:
            return node if node.stem == stem else None
        if cur_depth >= self.N:
            return None
        c = node.children.get(stem[cur_depth])
        return None if c is None else self._get_stem(c, stem, cur_depth + 1)

    def get_single(self, key):  # lib.rs:118-125
        e = self._get_stem(self.root, tuple(key), 0)
        return None if e is None else e.leaves.get(key[-1])

    def path_to_stem(self, key):  # node.rs:97-120 -> [(prefix, unit)]
        path, node = [], self.root
        while not node.ext:
            d = len(path)
            if d >= self.N or key[d] not in node.children:
                raise KeyError("InvalidPath")
            path.append((tuple(key[:d + 1]), key[d]))
            node = node.children[key[d]]
        return path

    # node.rs:205-277
    def _gen(self, node, commit):
        N = self.N
        if node.has_commit:
            return node.commit
        if node.ext:
            c1 = [0] * N
            c2 = [0] * N
            for index, leaf in node.leaves.items():
                low, high = _split(leaf)
                il, ih = (2 * index) % N, (2 * index + 1) % N
                if index < N // 2:
                    c1[il], c1[ih] = low, high
                else:
                    c2[il], c2[ih] = low, high
            C1, C2 = commit(c1), commit(c2)
            stem_item = int.from_bytes(bytes(node.stem), "little") % R  # bytes_to_item(stem.to_bytes())
            node.commit = commit([1, stem_item, to_data_item(C1), to_data_item(C2)])
        else:
            vec = [0] * 256
            for k, child in node.children.items():
                vec[k] = to_data_item(self._gen(child, commit))
            node.commit = commit(vec)
        node.has_commit = True
        return node.commit

    def commitment(self, commit):  # lib.rs:127-129
        return self._gen(self.root, commit)
