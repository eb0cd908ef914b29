"""Writes tests/golden/format_vectors.json — the parity pins for this path.

The reference (ikanago/horreum) is Rust and cannot be built or run in this
container (no cargo/rustc, crates not vendored), so these fixtures are the
known-answer vectors its own unit tests assert, transcribed as data: inputs
(pairs, stride, keys) and expected outputs (bytes, blocks, lookups, merge
results).  Each case names the reference test (file:line) it comes from.

Run:  python tests/golden/make_golden.py   (rewrites the JSON next to it)
"""
import json
import os


def b(s):
    return s.encode("utf-8") if isinstance(s, str) else bytes(s)


def hx(x):
    return None if x is None else b(x).hex()


def pairs(lst):
    return [[hx(k), hx(v)] for k, v in lst]


P16 = [  # src/sstable/index.rs:87-104 (also table.rs:113-130)
    ("abc00", "def"), ("abc01", "defg"), ("abc02", "de"), ("abc03", "defgh"),
    ("abc04", "defg"), ("abc05", "defghij"), ("abc06", "def"), ("abc07", "defgh"),
    ("abc08", None), ("abc09", None), ("abc10", None), ("abc11", None),
    ("abc12", None), ("abc13", None), ("abc14", None), ("abc15", None),
]

cases = {
    # ---- src/format.rs ----------------------------------------------------
    "serialize": {  # src/format.rs:90-97
        "ref": "src/format.rs:90-97",
        "pairs": pairs([("abc", "defg")]),
        "bytes": bytes([3, 0, 0, 0, 0, 0, 0, 0, 4, 0, 0, 0, 0, 0, 0, 0,
                        97, 98, 99, 100, 101, 102, 103]).hex(),
    },
    "serialize_lacking_value": {  # src/format.rs:99-106
        "ref": "src/format.rs:99-106",
        "pairs": pairs([("abc", None)]),
        "bytes": bytes([3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                        97, 98, 99]).hex(),
    },
    "serialize_non_ascii": {  # src/format.rs:108-119
        "ref": "src/format.rs:108-119",
        "pairs": pairs([("日本語💖", "ржавчина")]),
        "bytes": bytes([
            13, 0, 0, 0, 0, 0, 0, 0, 16, 0, 0, 0, 0, 0, 0, 0, 230, 151, 165, 230, 156, 172,
            232, 170, 158, 240, 159, 146, 150, 209, 128, 208, 182, 208, 176, 208, 178, 209,
            135, 208, 184, 208, 189, 208, 176,
        ]).hex(),
    },
    "serialize_flatten": {  # src/format.rs:121-136
        "ref": "src/format.rs:121-136",
        "pairs": pairs([("abc00", "def"), ("abc01", "defg"), ("abc02", "de")]),
        "bytes": bytes([
            5, 0, 0, 0, 0, 0, 0, 0, 3, 0, 0, 0, 0, 0, 0, 0, 97, 98, 99, 48, 48, 100, 101, 102,
            5, 0, 0, 0, 0, 0, 0, 0, 4, 0, 0, 0, 0, 0, 0, 0, 97, 98, 99, 48, 49, 100, 101, 102,
            103, 5, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 0, 0, 0, 97, 98, 99, 48, 50, 100, 101,
        ]).hex(),
    },
    "deserialize": {  # src/format.rs:138-150
        "ref": "src/format.rs:138-150",
        "bytes": bytes([3, 0, 0, 0, 0, 0, 0, 0, 4, 0, 0, 0, 0, 0, 0, 0,
                        97, 98, 99, 100, 101, 102, 103]).hex(),
        "pairs": pairs([("abc", "defg")]),
    },
    "deserialize_lacking_value": {  # src/format.rs:152-158
        "ref": "src/format.rs:152-158",
        "bytes": bytes([3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 97, 98, 99]).hex(),
        "pairs": pairs([("abc", None)]),
    },
    "deserialize_non_ascii": {  # src/format.rs:160-175
        "ref": "src/format.rs:160-175",
        "bytes": bytes([
            13, 0, 0, 0, 0, 0, 0, 0, 16, 0, 0, 0, 0, 0, 0, 0, 230, 151, 165, 230, 156, 172, 232,
            170, 158, 240, 159, 146, 150, 209, 128, 208, 182, 208, 176, 208, 178, 209, 135, 208,
            184, 208, 189, 208, 176,
        ]).hex(),
        "pairs": pairs([("日本語💖", "ржавчина")]),
    },
    "ordering": {  # src/format.rs:177-183: derived Ord, key bytes first
        "ref": "src/format.rs:177-183",
        "less": pairs([("abc", "defg")]),
        "greater": pairs([("日本語💖", "ржавчина")]),
    },
    "deserialize_from_bytes": {  # src/format.rs:185-200 (round trip)
        "ref": "src/format.rs:185-200",
        "pairs": pairs([("abc00", "def"), ("abc01", "defg"), ("abc02", "de"),
                        ("abc03", "defgh")]),
    },
    # ---- src/sstable/storage.rs -------------------------------------------
    "storage_read": {  # src/sstable/storage.rs:78-95 (file bytes incl. tombstone)
        "ref": "src/sstable/storage.rs:78-95",
        "pairs": pairs([("abc00", "def"), ("abc01", None)]),
        "bytes": bytes([
            5, 0, 0, 0, 0, 0, 0, 0, 3, 0, 0, 0, 0, 0, 0, 0, 97, 98, 99, 48, 48, 100, 101, 102,
            5, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 97, 98, 99, 48, 49,
        ]).hex(),
    },
    "storage_read_all": {  # src/sstable/storage.rs:97-107 (round trip)
        "ref": "src/sstable/storage.rs:97-107",
        "pairs": pairs([("abc00", "def"), ("abc01", "xxx"), ("abc02", None)]),
    },
    # ---- src/sstable/index.rs ---------------------------------------------
    "index_creation": {  # src/sstable/index.rs:85-117
        "ref": "src/sstable/index.rs:85-117",
        "pairs": pairs(P16),
        "stride": 3,
        # (first key, position, length)
        "blocks": [[hx("abc00"), 0, 72], [hx("abc03"), 72, 79], [hx("abc06"), 151, 71],
                   [hx("abc09"), 222, 63], [hx("abc12"), 285, 63], [hx("abc15"), 348, 21]],
    },
    "index_get": {  # src/sstable/index.rs:119-144
        "ref": "src/sstable/index.rs:119-144",
        "pairs": pairs(P16),
        "stride": 3,
        "lookups": [[hx("a"), None], [hx("abc01"), [0, 72]], [hx("abc03"), [72, 79]],
                    [hx("abc15"), [348, 21]]],
    },
    # ---- src/sstable/table.rs ---------------------------------------------
    "table_create": {  # src/sstable/table.rs:93-108: file == serialize_flatten,
        # with a duplicate key and an out-of-order tombstone, stride 1
        "ref": "src/sstable/table.rs:93-108",
        "pairs": pairs([("abc", "defg"), ("abc", None), ("日本語💖", "ржавчина")]),
        "stride": 1,
    },
    "table_search": {  # src/sstable/table.rs:110-144: block-local get
        "ref": "src/sstable/table.rs:110-144",
        "pairs": pairs(P16),
        "stride": 3,
        "gets": [[hx("abc04"), [hx("abc04"), hx("defg")]],
                 [hx("abc15"), [hx("abc15"), None]],
                 [hx("abc011"), None], [hx("abc16"), None]],
    },
    "table_iterate": {  # src/sstable/table.rs:146-168
        "ref": "src/sstable/table.rs:146-168",
        "pairs": pairs([("abc00", "def"), ("abc01", "defg"), ("abc02", None)]),
        "stride": 3,
    },
    "table_open_existing": {  # src/sstable/table.rs:170-185
        "ref": "src/sstable/table.rs:170-185",
        "pairs": pairs([("abc00", "def"), ("abc01", "defg"), ("abc02", None)]),
        "stride": 3,
    },
    # ---- src/sstable/manager.rs -------------------------------------------
    "compaction": {  # src/sstable/manager.rs:327-358.  The test hands this list to
        # compact_inner as-is (:355-357), so iterator 0 here is the FIRST
        # iterator and wins ties (min_by_key keeps the first minimum).  In
        # production compact() builds the list newest table first (:148-151).
        "ref": "src/sstable/manager.rs:327-358",
        "iterators": [
            pairs([("abc02", "def"), ("abc04", "hoge"), ("abc05", None)]),
            pairs([("abc00", "xyz"), ("abc01", None)]),
            pairs([("abc00", "def"), ("abc01", "defg"), ("abc02", "xyz"), ("abc03", "defg")]),
        ],
        "expected": pairs([("abc00", "xyz"), ("abc01", None), ("abc02", "def"),
                           ("abc03", "defg"), ("abc04", "hoge"), ("abc05", None)]),
    },
    "manager_get_newest_first": {  # src/sstable/manager.rs:242-275 (tables 0..2)
        "ref": "src/sstable/manager.rs:242-275",
        "tables_oldest_first": [
            pairs([("abc00", "def"), ("abc01", "defg")]),
            pairs([("abc00", "xyz"), ("abc01", None)]),
            pairs([("abc02", "def")]),
        ],
        "stride": 2,
        "gets": [[hx("abc00"), [hx("abc00"), hx("xyz")]],
                 [hx("abc01"), [hx("abc01"), None]],
                 [hx("abc02"), [hx("abc02"), hx("def")]]],
    },
    "payload_size": {  # SSTable::open size = sum(klen + vlen): src/sstable/table.rs:36-45;
        # the sizes the manager tests pass to create() agree: 17, 13, 8, 5
        # (src/sstable/manager.rs:289, 298, 302, 305)
        "ref": "src/sstable/table.rs:36-45; src/sstable/manager.rs:283-306",
        "tables": [
            [pairs([("abc00", "def"), ("abc01", "defg")]), 17],
            [pairs([("abc00", "xyz"), ("abc01", None)]), 13],
            [pairs([("abc02", "def")]), 8],
            [pairs([("xxx", "42")]), 5],
        ],
    },
}


def main():
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "format_vectors.json")
    with open(out, "w", encoding="utf-8") as f:
        json.dump({"source": "ikanago/horreum unit tests (transcribed)", "cases": cases},
                  f, indent=1, ensure_ascii=False)
        f.write("\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
