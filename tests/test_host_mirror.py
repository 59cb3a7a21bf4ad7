"""Host-mirror logic that runs before any GPU call: TreeHash's error texts
(shared/ssz/hash_test.go:142-148) and type validation, which must match the
reference exactly and never reach the device."""
import pytest

from prysm_amd import ssz as S
from tests.ssz_types import to_ssz_type, to_value


def test_error_vectors_without_gpu(ref_vectors):
    errs = [v for v in ref_vectors["tree_hash"] if v["error"]]
    assert len(errs) == 4
    for vec in errs:
        with pytest.raises(S.HashError) as ei:
            S.tree_hash(to_value(vec["type"], vec["value"]), to_ssz_type(vec["type"]))
        assert str(ei.value) == vec["error"], vec["ref"]


def test_nested_unsupported_types():
    with pytest.raises(S.HashError) as ei:
        S.tree_hash(["a"], S.Slice(S.Unsupported("string")))
    assert str(ei.value) == ("hash error: failed to get ssz utils: type string is not serializable "
                             "for input type []string")
    st = S.Struct("ssz.bad", [("A", S.Uint(8)), ("B", S.Unsupported("int"))])
    with pytest.raises(S.HashError) as ei:
        S.tree_hash({"A": 1, "B": 2}, st)
    assert str(ei.value) == "hash error: failed to get ssz utils: type int is not serializable for input type ssz.bad"


def test_nil_inside_slice_reports_element_path():
    simple = S.Struct("ssz.simpleStruct", [("B", S.Uint(16)), ("A", S.Uint(8))])
    with pytest.raises(S.HashError) as ei:
        S.tree_hash([{"B": 1, "A": 2}, None], S.Slice(S.Ptr(simple)))
    assert str(ei.value) == ("hash error: failed to hash element of slice/array: nil is not supported "
                             "for input type []*ssz.simpleStruct")


def test_xxx_fields_are_skipped():
    st = S.Struct("pb.X", [("A", S.Uint(8)), ("XXX_sizecache", S.Unsupported("int32"))])
    assert [n for n, _ in st.hashed_fields()] == ["A"]
