"""Generates tests/golden/*.json.

Two kinds of fixture, kept apart:

* REFERENCE-PINNED (``reference_vectors.json``): inputs and expected outputs
  transcribed as data from the reference's own tests —
    shared/hashutil/hash_test.go:13-31        (3 Keccak-256 KATs)
    shared/ssz/hash_test.go:35-148            (54 TreeHash vectors + 4 errors)
    shared/ssz/hash_test.go:151-178           (4 merkleHash vectors)
    shared/ssz/example_and_test.go:105,144    (2 struct-hash vectors)
    shared/hashutil/merkleRoot_test.go:8-29   (4-leaf MerkleRoot, expected
                                               value derived by the test itself)
  Go types are written as the tuple model of oracle/ssz_ref.py.
* RESTATEMENT-DERIVED (``restatement_vectors.json``): outputs of the CPU
  oracle (oracle/*.c) on seeded synthetic inputs, for sizes and edge cases no
  reference vector covers (N > 10, upper-level 160-B odd pad, item sizes that
  do not divide 128, >=128-B items, deposit tries).  The oracle producing
  them is itself pinned by the first file (tests/test_oracle.py).

Run:  python tests/golden/make_golden.py   (needs only the C oracle).
"""
from __future__ import annotations

import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402

U8, U16, U32, U64 = ["uint", 8], ["uint", 16], ["uint", 32], ["uint", 64]
SIMPLE = ["struct", "ssz.simpleStruct", [["B", U16], ["A", U8]]]  # encode_test.go:313-316
INNER = ["struct", "ssz.innerStruct", [["V", U16]]]  # encode_test.go:318-320
OUTER = ["struct", "ssz.outerStruct", [["V", U8], ["SubV", INNER]]]  # :322-325
ARRAYS = ["struct", "ssz.arrayStruct", [["V", ["slice", SIMPLE]]]]  # :327-329
POINTER = ["struct", "ssz.pointerStruct", [["P", ["ptr", SIMPLE]], ["V", U8]]]  # :331-334
HASHABLE = ["hashable", "ssz.hashableInterfaceTest", "pad28_left"]  # hash_test.go:19-32


def _s(b, a):
    return {"B": b, "A": a}


def reference_vectors():
    # shared/hashutil/hash_test.go:13-31
    kats = [
        {"ref": "shared/hashutil/hash_test.go:13-14", "in": "00",
         "out": bytes([188, 54, 120, 158, 122, 30, 40, 20, 54, 70, 66, 41, 130, 143, 129, 125, 102, 18,
                       247, 180, 119, 214, 101, 145, 255, 150, 169, 224, 100, 188, 201, 138]).hex()},
        {"ref": "shared/hashutil/hash_test.go:19-20", "in": "01",
         "out": bytes([95, 231, 249, 119, 231, 29, 186, 46, 161, 166, 142, 33, 5, 123, 238, 187, 155, 226,
                       172, 48, 198, 65, 10, 163, 141, 79, 63, 190, 65, 220, 255, 210]).hex()},
        {"ref": "shared/hashutil/hash_test.go:26-27", "in": b"abc".hex(),
         "out": "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"},
    ]
    T = []  # shared/ssz/hash_test.go:35-148, in order

    def add(line, typ, val, out=None, err=None):
        T.append({"ref": f"shared/ssz/hash_test.go:{line}", "type": typ, "value": val,
                  "output": out.lower() if out else None, "error": err})

    z = "00" * 32
    add(37, ["bool"], False, z)
    add(38, ["bool"], True, "01" + "00" * 31)
    for line, (typ, vals) in zip((41, 48, 56, 65), (
            (U8, [0, 1, 16, 128, 255]),
            (U16, [0, 1, 16, 128, 255, 65535]),
            (U32, [0, 1, 16, 128, 255, 65535, 4294967295]),
            (U64, [0, 1, 16, 128, 255, 65535, 4294967295, 18446744073709551615]))):
        for i, v in enumerate(vals):
            enc = v.to_bytes(typ[1] // 8, "little")
            add(line + i, typ, v, (enc + b"\0" * 32)[:32].hex())
    add(75, ["bytes"], [], "E8E77626586F73B955364C7B4BBF0BB7F7685EBD40E852B164633A4ACBD3244C")
    add(76, ["bytes"], [1], "B2559FED89F0EC17542C216683DC6B75506F3754E0C045742936742CAE6343CA")
    add(77, ["bytes"], [1, 2, 3, 4, 5, 6], "1310542D28BE8E0B3FF72E985BC06232B9A30D93AE1AD2E33C5383A54AB5C9A7")
    add(80, ["slice", U16], [], "DFDED4ED5AC76BA7379CFE7B3B0F53E768DCA8D45A34854E649CFC3C18CBD9CD")
    add(81, ["slice", U16], [1], "E3F121F639DAE19B7E2FD6F5002F321B83F17288A7CA7560F81C2ACE832CC5D5")
    add(82, ["slice", U16], [1, 2], "A9B7D66D80F70C6DA7060C3DEDB01E6ED6CEA251A3247093CBF27A439ECB0BEA")
    add(83, ["slice", ["slice", U16]], [[1, 2, 3, 4], [5, 6, 7, 8]],
        "1A400EB17C755E4445C2C57DD2D3A0200A290C56CD68957906DD7BFE04493B10")
    add(89, ["bytearray", 1], [1], "B2559FED89F0EC17542C216683DC6B75506F3754E0C045742936742CAE6343CA")
    add(90, ["bytearray", 6], [1, 2, 3, 4, 5, 6], "1310542D28BE8E0B3FF72E985BC06232B9A30D93AE1AD2E33C5383A54AB5C9A7")
    add(91, ["array", U16, 1], [1], "E3F121F639DAE19B7E2FD6F5002F321B83F17288A7CA7560F81C2ACE832CC5D5")
    add(92, ["array", U16, 2], [1, 2], "A9B7D66D80F70C6DA7060C3DEDB01E6ED6CEA251A3247093CBF27A439ECB0BEA")
    add(93, ["array", ["array", U16, 4], 2], [[1, 2, 3, 4], [5, 6, 7, 8]],
        "1A400EB17C755E4445C2C57DD2D3A0200A290C56CD68957906DD7BFE04493B10")
    add(99, SIMPLE, _s(0, 0), "99FF0D9125E1FC9531A11262E15AEB2C60509A078C4CC4C64CEFDFB06FF68647")
    add(100, SIMPLE, _s(2, 1), "D2B49B00C76582823E30B56FE608FF030EF7B6BD7DCC16B8994C9D74860A7E1C")
    add(101, OUTER, {"V": 3, "SubV": {"V": 6}}, "BB2F30386C55445381EEE7A33C3794227B8C8E4BE4CAA54506901A4DDFE79EE2")
    add(107, ARRAYS, {"V": [_s(2, 1), _s(4, 3)]}, "F3032DCE4B4218187E34AA8B6EF87A3FABE1F8D734CE92796642DC6B2911277C")
    add(113, ["slice", OUTER], [{"V": 3, "SubV": {"V": 6}}, {"V": 5, "SubV": {"V": 7}}],
        "DE43BC05AA6B011121F9590C10DE1734291A595798C84A0E3EDD1CC1E6710908")
    add(119, ["ptr", SIMPLE], _s(2, 1), "D2B49B00C76582823E30B56FE608FF030EF7B6BD7DCC16B8994C9D74860A7E1C")
    add(120, POINTER, {"P": _s(2, 1), "V": 3}, "D365B04884AA7B9160F5E405796F0EB7521FC69BD79D934DA72EDA1FC98B5971")
    add(121, ["ptr", POINTER], {"P": _s(2, 1), "V": 3}, "D365B04884AA7B9160F5E405796F0EB7521FC69BD79D934DA72EDA1FC98B5971")
    add(122, ["ptr", ["bytes"]], [1, 2, 3, 4], "5C8046AB6A4E32E5C0017620A1844E5851074E4EDA685A920E8C70007E675E5C")
    add(123, ["ptr", ["slice", U64]], [1, 2], "2F3E7F86CF5B91C6FC45FDF54254DE256F4FFFE775F0217C876961C4211E5DC2")
    add(124, ["slice", ["ptr", SIMPLE]], [_s(2, 1), _s(4, 3)],
        "1D5CDF2C53DD8AC743E17E1A7A8B1CB6E615FA63EC915347B3E9ACFB58F89158")
    add(128, ["array", ["ptr", SIMPLE], 2], [_s(2, 1), _s(4, 3)],
        "1D5CDF2C53DD8AC743E17E1A7A8B1CB6E615FA63EC915347B3E9ACFB58F89158")
    add(132, ["slice", ["ptr", POINTER]], [{"P": _s(2, 1), "V": 0}, {"P": _s(4, 3), "V": 1}],
        "4AC9B9E64A067F6C007C3FE8116519D86397BDA1D9FBEDEEDF39E50D132669C7")
    add(138, HASHABLE, [0, 2, 4, 6], "0000000000000000000000000000000000000000000000000000000000020406")
    add(143, ["nil"], None, err="hash error: nil is not supported for input type <nil>")
    add(144, ["ptr", ["bytes"]], None, err="hash error: nil is not supported for input type *[]uint8")
    add(145, POINTER, {"P": None, "V": 0},
        err="hash error: failed to hash field of struct: nil is not supported for input type ssz.pointerStruct")
    add(148, ["string"], "abc", err="hash error: type string is not serializable for input type string")

    merkle = [  # shared/ssz/hash_test.go:151-178
        {"ref": "shared/ssz/hash_test.go:152", "items": [],
         "output": "DFDED4ED5AC76BA7379CFE7B3B0F53E768DCA8D45A34854E649CFC3C18CBD9CD".lower()},
        {"ref": "shared/ssz/hash_test.go:153", "items": ["0102", "0304"],
         "output": "64F741B8BAB62525A01F9084582C148FF56C82F96DC12E270D3E7B5103CF7B48".lower()},
        {"ref": "shared/ssz/hash_test.go:154-165", "items": [(bytes([i]) * 16).hex() for i in range(1, 11)],
         "output": "839D98509E2EFC53BD1DEA17403921A89856E275BBF4D56C600CC3F6730AAFFA".lower()},
        {"ref": "shared/ssz/hash_test.go:166-177", "items": [(bytes([i]) * 32).hex() for i in range(1, 11)],
         "output": "55DC6699E7B5713DD9102224C302996F931836C6DAE9A4EC6AB49C966F394685".lower()},
    ]
    examples = [  # struct-hash semantics (SURVEY.md §4 caveat on exampleStruct1's self-recursion)
        {"ref": "shared/ssz/example_and_test.go:105",
         "type": ["struct", "ssz.exampleStruct1", [["Field1", U8], ["Field2", ["bytes"]]]],
         "value": {"Field1": 10, "Field2": [1, 2, 3, 4]},
         "output": "898470f5d98653c8e4fb2c7ae771019402cca8ccaa71a9c2ea4ad129e3c431d0", "error": None},
        {"ref": "shared/ssz/example_and_test.go:144",
         "type": ["struct", "ssz.exampleStruct2Export", [["Field2", ["bytes"]]]],
         "value": {"Field2": [1, 2, 3, 4]},
         "output": "b982eb8cf7e1d6f5ec77f0ae4a9ed44bde23da284488f498176a5123fe05e7dd", "error": None},
    ]
    # merkleRoot_test.go:8-29 builds its expected root by hand from Hash().
    ha, hb, hc, hd = (O.keccak256(c) for c in (b"a", b"b", b"c", b"d"))
    mroot = O.keccak256(O.keccak256(ha + hb) + O.keccak256(hc + hd))
    merkle_root = [{"ref": "shared/hashutil/merkleRoot_test.go:8-29",
                    "values": [b"a".hex(), b"b".hex(), b"c".hex(), b"d".hex()], "output": mroot.hex()}]
    return {"keccak256_kats": kats, "tree_hash": T + examples, "merkle_hash": merkle,
            "merkle_root": merkle_root}


SEED0 = 0x5EED000000000000


def restatement_vectors():
    cases = []
    sizes = list(range(0, 71)) + [127, 128, 129, 255, 256, 257, 1000, 1023, 1024, 1025, 4099]
    for item_len in (32, 8, 1, 2, 4, 16, 64, 128, 3, 48, 96, 200, 280):
        for n in sizes:
            if item_len >= 128 and n > 300:
                continue
            seed = SEED0 + 100 + item_len
            items = O.splitmix_bytes(n * item_len, seed)
            root = O.merkle_hash_flat(items, n, item_len)
            cases.append({"n": n, "item_len": item_len, "seed": seed, "root": root.hex()})
    # Reference-shaped list vectors from SURVEY.md §8(c) (restatement cross-checks)
    lists = [
        {"items": [(bytes([i]) * 32).hex() for i in range(5)],
         "output": "a855f7cae37c69124892573be57123780de25b544bb3c4ef10e6b44d294d67e2"},
        {"items": [(bytes([i]) * 32).hex() for i in range(20)],
         "output": "079e9bbb8b2d10b2b83b3466e85909f5f87e6f8caec83a4c835be01a234b49fb"},
        {"items": [(bytes([i]) * 32).hex() for i in range(33)],
         "output": "ed10886562a707c20bec33e6db1f5ea350646a84cb333b8c16c4f72e2e3e2dbc"},
        {"items": [O.keccak256(struct.pack("<Q", i)).hex() for i in range(1024)],
         "output": "8c54505db52ffb0604bac428fc59d10fc99a7798138b6d1ba8ee6be6038e1111"},
    ]
    for l in lists:
        got = O.merkle_hash([bytes.fromhex(x) for x in l["items"]]).hex()
        assert got == l["output"], (got, l["output"])
    # Deposit tries: deposits of 280 B (block.go:103-130 layout) and short ones
    tries = []
    for n in (0, 1, 2, 3, 5, 8, 33, 1000):
        seed = SEED0 + 5
        deps = [bytes(O.splitmix_bytes(280, seed, 35 * i)) for i in range(n)]
        root, _ = O.deposit_trie_levels(deps)
        tries.append({"n": n, "deposit_len": 280, "seed": seed, "word_stride": 35, "root": root.hex()})
    # Synthetic-stream digests (pins the device SplitMix64 generator)
    stream = {"seed": SEED0 + 2, "words": [O.lib().or_splitmix64_word(SEED0 + 2, k) for k in range(8)]}
    return {"merkle_flat": cases, "merkle_lists": lists, "deposit_tries": tries, "splitmix": stream}


def main():
    ref = reference_vectors()
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(ref, f, indent=1)
    res = restatement_vectors()
    with open(os.path.join(HERE, "restatement_vectors.json"), "w") as f:
        json.dump(res, f, indent=0)
    print("wrote", len(ref["tree_hash"]), "tree-hash vectors,", len(res["merkle_flat"]), "merkle cases")


if __name__ == "__main__":
    main()
