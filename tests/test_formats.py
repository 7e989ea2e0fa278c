"""Persisted formats: QuantizedTensor Codable JSON
(GEMMQuantization.swift:906-1077), QuantizationParameters / QuantizationMode encodings
(:43-99, :212-273) and MaskingCalibration JSON + store (MaskingStrategyHeuristic.swift:152-191,
:415-447).  CPU only (tensors on the host); the GPU round trip through the quantised attention
is tests/test_formats_gpu.py.

The reference commits no serialized files; the fixture below is written by hand in the shape
Swift's JSONEncoder produces for these Codable types (prettyPrinted: two-space indent,
"key" : value; Data as base64), so decoding it pins field names, nesting and defaults."""
import base64
import json

import numpy as np
import pytest
import torch

import mfa_amd as mfa
import mfa_formats as F
import oracle_lib as ol

P = mfa.Precision

SWIFT_STYLE_FIXTURE = """{
  "data" : "%s",
  "header" : {
    "dtype" : "INT8",
    "elementCount" : 6,
    "hasBlockScales" : false,
    "hasBlockZeroPoints" : false,
    "hasPrecomputedSums" : false,
    "quantMode" : {
      "caseName" : "tensorWise"
    },
    "shape" : [
      2,
      3
    ],
    "version" : 1
  },
  "parameters" : {
    "mode" : {
      "caseName" : "tensorWise"
    },
    "precision" : 3,
    "scale" : 0.015625,
    "zeroPoint" : 0
  }
}""" % base64.b64encode(bytes([0, 1, 127, 0x81, 0xFF, 64, 0, 0])).decode()


def test_mode_json():
    assert F.QuantizationMode.tensor_wise().to_json() == {"caseName": "tensorWise"}
    assert F.QuantizationMode.row_wise().to_json() == {"caseName": "rowWise"}
    assert F.QuantizationMode.blockwise(64, True).to_json() == {
        "caseName": "blockwise", "blockSize": 64, "bothOperands": True}
    # bothOperands is decodeIfPresent (default false)
    m = F.QuantizationMode.from_json({"caseName": "blockwise", "blockSize": 32})
    assert (m.case, m.block_size_k, m.both_operands) == ("blockwise", 32, False)
    with pytest.raises(F.FormatError):
        F.QuantizationMode.from_json({"caseName": "columnWise"})


def test_parameters_json_and_defaults():
    p = F.QuantizationParameters.from_arrays([0.5, 0.25, 0.125], [0, 0, 0], P.INT8,
                                             F.QuantizationMode.blockwise(8), F.STRATEGY_SYMMETRIC)
    j = p.to_json()
    assert list(j) == ["scale", "zeroPoint", "precision", "mode", "additionalScales",
                       "additionalZeroPoints", "strategy", "strategyVersion"]
    assert j["additionalScales"] == [0.25, 0.125] and j["strategy"] == 2
    q = F.QuantizationParameters.from_json(j)
    assert q.all_scales == [0.5, 0.25, 0.125]
    # strategy / strategyVersion absent: legacy / current (init(from:) :240-245); optional
    # arrays absent: omitted on encode (encodeIfPresent, :269-270).
    q = F.QuantizationParameters.from_json({"scale": 1.0, "zeroPoint": 3, "precision": 3,
                                            "mode": {"caseName": "tensorWise"}})
    assert (q.strategy, q.strategy_version, q.zero_point) == (0, 1, 3)
    assert "additionalScales" not in q.to_json()


def test_parameters_validation():
    # validate (:181-210): symmetric needs zero zero-points and blockwise sizes % 8 == 0.
    with pytest.raises(F.FormatError, match="zero points to be zero"):
        F.QuantizationParameters(1.0, 2, P.INT8, strategy=F.STRATEGY_SYMMETRIC)
    with pytest.raises(F.FormatError, match="multiples of 8"):
        F.QuantizationParameters(1.0, 0, P.INT4, F.QuantizationMode.blockwise(12),
                                 strategy=F.STRATEGY_SYMMETRIC)
    F.QuantizationParameters(1.0, 2, P.FP16, strategy=F.STRATEGY_SYMMETRIC)  # not quantized: ok


def test_decode_swift_style_fixture():
    r = F.QuantizedTensorRecord.decode(SWIFT_STYLE_FIXTURE.encode(), device="cpu")
    assert r.element_count == 6 and r.original_shape == [2, 3]
    assert r.parameters.precision == P.INT8 and r.parameters.scale == 0.015625
    assert r.block_size_k is None and r.block_scales is None
    # The buffer keeps its full (64-byte-rounded in the reference) length.
    assert r.data.tolist() == [0, 1, 127, 0x81, 0xFF, 64, 0, 0]
    q = r.data.numpy()[:6].view(np.int8)
    vals = ol.dequantize(q, 6, int(P.INT8), 0.015625, 0) if hasattr(ol, "dequantize") else \
        q.astype(np.float32) * np.float32(0.015625)
    assert np.array_equal(vals, np.array([0, 1, 127, -127, -1, 64], np.float32) * np.float32(0.015625))


def test_record_round_trip_blockwise():
    rng = np.random.default_rng(0)
    data = torch.from_numpy(rng.integers(0, 256, 40, dtype=np.uint8))
    sc = torch.tensor([0.5, 0.25, 0.125, 2.0], dtype=torch.float32)
    zp = torch.zeros(4, dtype=torch.int32)
    params = F.QuantizationParameters.from_arrays(sc.tolist(), zp.tolist(), P.INT4,
                                                  F.QuantizationMode.blockwise(8), F.STRATEGY_SYMMETRIC)
    r = F.QuantizedTensorRecord(data, params, 80, [16, 5], sc, zp, 8)
    obj = json.loads(r.encode())
    assert obj["header"]["blockSizeK"] == 8 and obj["header"]["hasBlockScales"]
    assert obj["header"]["dtype"] == "INT4"
    assert np.frombuffer(base64.b64decode(obj["blockScales"]), np.float32).tolist() == sc.tolist()
    s = F.QuantizedTensorRecord.decode(r.encode(), device="cpu")
    assert torch.equal(s.data, data) and torch.equal(s.block_scales, sc)
    assert torch.equal(s.block_zero_points, zp) and s.block_size_k == 8
    assert s.parameters == params


def test_record_errors():
    obj = json.loads(SWIFT_STYLE_FIXTURE)
    obj["header"]["version"] = 2
    with pytest.raises(F.FormatError, match="Unsupported serialization version: 2"):
        F.QuantizedTensorRecord.from_json_obj(obj, device="cpu")
    obj = json.loads(SWIFT_STYLE_FIXTURE)
    obj["header"]["elementCount"] = 9
    with pytest.raises(F.FormatError, match="bytes"):
        F.QuantizedTensorRecord.from_json_obj(obj, device="cpu")


def test_row_wise_record_rebuilds_scales():
    params = F.QuantizationParameters.from_arrays([0.5, 0.25], [0, 0], P.INT8,
                                                  F.QuantizationMode.row_wise())
    r = F.QuantizedTensorRecord(torch.zeros(8, dtype=torch.uint8), params, 8, [2, 4])
    obj = json.loads(r.encode())
    assert "blockSizeK" not in obj["header"] and not obj["header"]["hasBlockScales"]
    s = F.QuantizedTensorRecord.decode(r.encode(), device="cpu")
    assert s.block_scales.tolist() == [0.5, 0.25]


def test_masking_calibration_store(tmp_path):
    cal = F.MaskingCalibration("AMD Instinct MI355X", [
        F.MaskingCalibrationEntry(4096, 128, "bitmask", 0.25, 0.5),
        F.MaskingCalibrationEntry(512, 64, "elementWise", 0.125, 0.0625)])
    url = F.MaskingCalibrationStore.default_url("AMD Instinct MI355X")
    assert url.name == "AMD_Instinct_MI355X.json"
    assert url.parts[-3:] == ("FlashAttention", "masking-calibration", "AMD_Instinct_MI355X.json")
    path = tmp_path / "sub" / "cal.json"
    F.MaskingCalibrationStore.save(cal, path)
    text = path.read_text()
    assert text.startswith('{\n  "deviceName" : "AMD Instinct MI355X",\n  "entries" : [')
    assert F.MaskingCalibrationStore.load(path) == cal
    with pytest.raises(F.FormatError):
        F.MaskingCalibration.from_json({"deviceName": "x", "entries": [{"strategy": "other"}]})


def test_heuristic_apply_overrides_default_rule():
    h = F.MaskingStrategyHeuristic.shared
    h.reset()
    base = h.recommend(4000, 128)
    other = "elementWise" if base == "bitmask" else "bitmask"
    h.apply(F.MaskingCalibration("dev", [F.MaskingCalibrationEntry(4096, 128, other, 1.0, 2.0)]))
    assert h.recommend(4000, 128) == other          # 4000 falls in the 4096 bucket
    assert h.recommend(4000, 64) == F.MaskingStrategyHeuristic().recommend(4000, 64)
    h.reset()
    assert h.recommend(4000, 128) == base
