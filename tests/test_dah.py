"""DataAvailabilityHeader conversions and ValidateBasic.

Mirrors /root/reference/pkg/da/data_availability_header_test.go:
  * TestDataAvailabilityHeaderProtoConversion (:101-133): min and max (k=128)
    DAH through ToProto -> DataAvailabilityHeaderFromProto are equal; here
    also through the protobuf wire bytes of
    proto/celestia/core/v1/da/data_availability_header.proto:16-21;
  * Test_DAHValidateBasic (:135-215): min / max pass; too big, too small,
    bad hash and mismatched root counts fail with the reference's messages;
  * TestSquareSize (:217-245).
The wire format and the size checks are host logic (CPU); everything that
hashes roots runs on the GPU (libcda.so).
"""
import pytest

import pyref
from celestia_da import da

ROOT = bytes(range(90))


def test_marshal_wire_layout():
    dah = da.DataAvailabilityHeader([b"\x01" * 90, b"\x02" * 90], [b"\x03" * 90])
    wire = dah.marshal()
    # field 1 (wire type 2) = 0x0a, length 90 = 0x5a; field 2 = 0x12
    assert wire == (b"\x0a\x5a" + b"\x01" * 90 + b"\x0a\x5a" + b"\x02" * 90 + b"\x12\x5a" + b"\x03" * 90)
    p = da.unmarshal_data_availability_header(wire)
    assert p == dah.to_proto()


def test_unmarshal_long_roots_and_unknown_fields():
    big = bytes(300)                       # two-byte varint length
    dah = da.DataAvailabilityHeader([big], [ROOT])
    wire = dah.marshal()
    assert wire[:3] == b"\x0a\xac\x02"
    extra = b"\x18\x96\x01" + b"\x25\x00\x00\x00\x00"   # unknown varint + fixed32 fields
    p = da.unmarshal_data_availability_header(extra + wire)
    assert p == {"row_roots": [big], "column_roots": [ROOT]}
    assert da.unmarshal_data_availability_header(b"") == {"row_roots": [], "column_roots": []}


@pytest.mark.parametrize("bad", [b"\x0a\x5a" + ROOT[:10], b"\x0a", b"\x08\x01", b"\x00\x01", b"\x0f"])
def test_unmarshal_malformed(bad):
    with pytest.raises(ValueError):
        da.unmarshal_data_availability_header(bad)


def test_validate_basic_size_errors():
    # the size checks run before any hashing (:134-162)
    maxw = da.MAX_EXTENDED_SQUARE_WIDTH
    too_big = da.DataAvailabilityHeader([b"\x01" * 32] * (maxw + 1), [b"\x01" * 32] * (maxw + 1))
    with pytest.raises(ValueError, match="maximum valid DataAvailabilityHeader has at most"):
        too_big.validate_basic()
    too_small = da.DataAvailabilityHeader([b"\x02" * 32], [b"\x02" * 32])
    with pytest.raises(ValueError, match="minimum valid DataAvailabilityHeader has at least"):
        too_small.validate_basic()
    mismatch = da.DataAvailabilityHeader([ROOT] * 2, [ROOT] * 3)
    with pytest.raises(ValueError, match="unequal number of row and column roots"):
        mismatch.validate_basic()
    with pytest.raises(ValueError, match="nil DataAvailabilityHeader"):
        da.data_availability_header_from_proto(None)


@pytest.mark.gpu
def test_validate_basic_bad_hash(ctx):
    dah = da.min_data_availability_header()
    dah.validate_basic()
    dah._hash = bytes([1, 2, 3, 4])
    with pytest.raises(ValueError, match="wrong hash"):
        dah.validate_basic()


@pytest.mark.gpu
def test_proto_conversion_min_max(ctx):
    shares = pyref.constant_shares(128 * 128)      # generateShares(maxSize), :247-263 shape
    big = da.new_data_availability_header(da.extend_shares(shares))
    big.validate_basic()
    # TestSquareSize (:217-245): min -> 1, max -> DefaultSquareSizeUpperBound
    assert da.min_data_availability_header().square_size() == 1
    assert big.square_size() == da.DEFAULT_SQUARE_SIZE_UPPER_BOUND
    for dah in (da.min_data_availability_header(), big):
        res = da.data_availability_header_from_proto(dah.to_proto())
        assert res.row_roots == dah.row_roots and res.column_roots == dah.column_roots
        assert res.hash() == dah.hash()
        wire = da.data_availability_header_from_proto(da.unmarshal_data_availability_header(dah.marshal()))
        assert wire.row_roots == dah.row_roots and wire.column_roots == dah.column_roots
        assert wire.hash() == dah.hash()


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols,size", [(6, 6, 90), (3, 5, 90), (4, 4, 33), (1, 0, 90), (2, 2, 0)])
def test_hash_any_shape_on_gpu(ctx, rows, cols, size):
    """Hash() is merkle.HashFromByteSlices(rowRoots || colRoots) for ANY
    slices (data_availability_header.go:92-108): a header decoded from the
    wire with 6 rows, unequal counts or other root sizes hashes like the
    reference (cda_merkle_root) instead of failing."""
    import numpy as np
    rng = np.random.default_rng(rows * 100 + cols * 10 + size)
    r = [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(rows)]
    c = [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(cols)]
    dah = da.DataAvailabilityHeader(r, c)
    assert dah.hash() == pyref.merkle_root(r + c)


@pytest.mark.gpu
def test_from_proto_six_roots_on_gpu(ctx):
    """DataAvailabilityHeaderFromProto of a 6 x 6 header: ValidateBasic passes
    (2 <= 6 <= 256, equal counts) and Hash() is the RFC-6962 root over 12
    items (split 8 | 4)."""
    r = [bytes([i]) * 90 for i in range(6)]
    c = [bytes([0x80 + i]) * 90 for i in range(6)]
    d = da.data_availability_header_from_proto({"row_roots": r, "column_roots": c})
    assert d.hash() == pyref.merkle_root(r + c)


def test_batch_shape_from_array_shape():
    """da._batch_shape: k comes from the array's shape, never
    rounded; an empty batch is (0, k); a non-square shape is an error."""
    import numpy as np
    from celestia_da import da as cda
    assert cda._batch_shape(np.zeros((3, 64, 512), np.uint8)) == (3, 8)
    assert cda._batch_shape(np.zeros((2, 16, 16, 512), np.uint8)) == (2, 16)
    assert cda._batch_shape(np.zeros((0, 16, 512), np.uint8)) == (0, 4)
    for bad in ((3, 60, 512), (2, 8, 4, 512), (2, 64, 256)):
        try:
            cda._batch_shape(np.zeros(bad, np.uint8))
        except ValueError:
            continue
        raise AssertionError(bad)
