"""Persisted formats of the reference, read and written by the MI355X library's host side.

* QuantizedTensor's Codable JSON (GEMM/GEMMQuantization.swift:906-1077) with its
  QuantizationParameters (:101-279) and QuantizationMode (:24-99) encodings: keyed objects
  under "header", "parameters", "data", "blockScales", "blockZeroPoints", "precomputedSums";
  buffers as base64 strings (JSONEncoder's default Data strategy).  The tensor's buffers live
  in HBM: encode copies them to the host, decode uploads them to the device again.
* MaskingCalibration JSON and MaskingCalibrationStore (Attention/MaskingStrategyHeuristic.swift:
  152-191, :415-447), plus the heuristic's in-memory cache that `apply` hydrates
  (:138-149) in front of the library's default rule (mfa_masking_default_rule).

Swift's JSONEncoder output is matched field for field (names, nesting, optional keys omitted
when nil, enums as their raw values).  Byte-for-byte layout (whitespace, number spelling)
is not a contract of the reference either: its decoder accepts any JSON spelling.
"""
from __future__ import annotations

import base64
import dataclasses
import json
import os
import pathlib
import threading
from typing import Optional

import mfa_amd as mfa

P = mfa.Precision
# String(describing: GEMMOperandPrecision) = the case name (GEMMOperandPrecision.swift:22-27).
PRECISION_NAME = {P.FP32: "FP32", P.FP16: "FP16", P.BF16: "BF16", P.INT8: "INT8", P.INT4: "INT4"}
SERIALIZATION_VERSION = 1            # SerializationHeader.currentVersion (:920)
STRATEGY_VERSION = 1                 # QuantizationStrategy.currentVersion (:41)
STRATEGY_LEGACY, STRATEGY_ASYMMETRIC, STRATEGY_SYMMETRIC = 0, 1, 2


class FormatError(ValueError):
    """DecodingError.dataCorrupted / preconditionFailure of the reference decoders."""


# ------------------------------------------------------------------------------ modes
@dataclasses.dataclass(frozen=True)
class QuantizationMode:
    """QuantizationMode (GEMMQuantization.swift:24-33); JSON per its Codable extension
    (:43-99): {"caseName": ..., "blockSize": k, "bothOperands": b} for blockwise."""
    case: str = "tensorWise"          # tensorWise | blockwise | rowWise
    block_size_k: int = 128           # QuantizationMode.defaultBlockSizeK (:32)
    both_operands: bool = False

    @staticmethod
    def tensor_wise():
        return QuantizationMode("tensorWise")

    @staticmethod
    def blockwise(block_size_k: int = 128, both_operands: bool = False):
        return QuantizationMode("blockwise", block_size_k, both_operands)

    @staticmethod
    def row_wise():
        return QuantizationMode("rowWise")

    def to_json(self) -> dict:
        if self.case == "blockwise":
            return {"caseName": "blockwise", "blockSize": self.block_size_k,
                    "bothOperands": self.both_operands}
        return {"caseName": self.case}

    @staticmethod
    def from_json(obj: dict) -> "QuantizationMode":
        name = obj.get("caseName")
        if name == "tensorWise":
            return QuantizationMode.tensor_wise()
        if name == "rowWise":
            return QuantizationMode.row_wise()
        if name == "blockwise":
            if "blockSize" not in obj:
                raise FormatError("blockwise mode without blockSize")
            return QuantizationMode.blockwise(int(obj["blockSize"]), bool(obj.get("bothOperands", False)))
        raise FormatError(f"unknown QuantizationMode caseName {name!r}")

    @property
    def abi(self) -> mfa.QuantMode:
        return {"tensorWise": mfa.QuantMode.tensorWise, "blockwise": mfa.QuantMode.blockwise,
                "rowWise": mfa.QuantMode.rowWise}[self.case]


# ------------------------------------------------------------------------- parameters
def _requires_params(prec: P) -> bool:
    return prec in (P.INT8, P.INT4)  # GEMMOperandPrecision.requiresQuantizationParameters


@dataclasses.dataclass
class QuantizationParameters:
    """QuantizationParameters (GEMMQuantization.swift:101-279).  For several scales (blockwise,
    row-wise) the first is `scale` and the rest `additional_scales` (:154-175)."""
    scale: float
    zero_point: int
    precision: P
    mode: QuantizationMode = dataclasses.field(default_factory=QuantizationMode)
    additional_scales: Optional[list] = None
    additional_zero_points: Optional[list] = None
    strategy: int = STRATEGY_LEGACY
    strategy_version: int = STRATEGY_VERSION

    def __post_init__(self):
        self.validate()

    @staticmethod
    def from_arrays(scales, zero_points, precision, mode, strategy=STRATEGY_LEGACY):
        scales = [float(s) for s in scales]
        zps = [int(z) for z in zero_points]
        return QuantizationParameters(
            scales[0] if scales else 1.0, zps[0] if zps else 0, precision, mode,
            scales[1:] if len(scales) > 1 else None, zps[1:] if len(zps) > 1 else None, strategy)

    @property
    def all_scales(self) -> list:
        return [self.scale] + list(self.additional_scales or [])

    @property
    def all_zero_points(self) -> list:
        return [self.zero_point] + list(self.additional_zero_points or [])

    def validate(self):
        """QuantizationParameters.validate (:181-210)."""
        if not _requires_params(P(self.precision)) or self.strategy != STRATEGY_SYMMETRIC:
            return
        nz = [z for z in self.all_zero_points if z != 0]
        if nz:
            raise FormatError(f"Symmetric quantization requires zero points to be zero; found {nz[0]}.")
        if self.mode.case == "blockwise" and self.mode.block_size_k % 8 != 0:
            raise FormatError("Symmetric block-wise quantization requires block sizes that are "
                              "multiples of 8.")

    def to_json(self) -> dict:
        """encode(to:) (:264-273): optional arrays only when present."""
        out = {"scale": float(self.scale), "zeroPoint": int(self.zero_point),
               "precision": int(self.precision), "mode": self.mode.to_json()}
        if self.additional_scales is not None:
            out["additionalScales"] = [float(s) for s in self.additional_scales]
        if self.additional_zero_points is not None:
            out["additionalZeroPoints"] = [int(z) for z in self.additional_zero_points]
        out["strategy"] = int(self.strategy)
        out["strategyVersion"] = int(self.strategy_version)
        return out

    @staticmethod
    def from_json(obj: dict) -> "QuantizationParameters":
        """init(from:) (:226-262): strategy defaults to legacy, strategyVersion to current."""
        try:
            return QuantizationParameters(
                float(obj["scale"]), int(obj["zeroPoint"]), P(int(obj["precision"])),
                QuantizationMode.from_json(obj["mode"]),
                obj.get("additionalScales"), obj.get("additionalZeroPoints"),
                int(obj.get("strategy", STRATEGY_LEGACY)),
                int(obj.get("strategyVersion", STRATEGY_VERSION)))
        except KeyError as e:
            raise FormatError(f"QuantizationParameters: missing key {e}") from None


# --------------------------------------------------------------------- quantized tensor
@dataclasses.dataclass
class QuantizedTensorRecord:
    """QuantizedTensor (GEMMQuantization.swift:680-718) over device tensors: `data` holds
    the quantised bytes (INT8, or INT4 packed two per byte), block scales / zero points are
    FP32 / INT32 device arrays (blockwise: one per block; row-wise: one per row)."""
    data: object                       # torch.uint8 device tensor
    parameters: QuantizationParameters
    element_count: int
    original_shape: list
    block_scales: object = None        # torch.float32 device tensor
    block_zero_points: object = None  # torch.int32 device tensor
    block_size_k: Optional[int] = None
    precomputed_sums: object = None    # device tensor (opaque bytes)

    # -- construction from the GPU quantiser
    @staticmethod
    def quantize(x, precision: P = P.INT8, mode: QuantizationMode = None,
                 strategy=STRATEGY_SYMMETRIC, stream=None) -> "QuantizedTensorRecord":
        """QuantizedTensor.from (:720-860) with the quantisation on the GPU (mfa_quantize).
        x: FP32/FP16/BF16 device tensor; 2-D view [shape[0], rest] for blockwise/row-wise."""
        import torch
        mode = mode or QuantizationMode.tensor_wise()
        shape = list(x.shape)
        rows = shape[0] if len(shape) >= 2 else 1
        cols = x.numel() // max(rows, 1)
        bs = mode.block_size_k if mode.case == "blockwise" else 0
        data, scale, bsc, bzp = mfa.quantize(x, precision, mode.abi, rows=rows, cols=cols,
                                             block_size=bs, stream=stream)
        torch.cuda.synchronize()
        if mode.case == "tensorWise":
            params = QuantizationParameters(float(scale.item()), 0, precision, mode, strategy=strategy)
            return QuantizedTensorRecord(data, params, x.numel(), shape)
        scales = bsc.cpu().tolist()
        zps = bzp.cpu().tolist()
        params = QuantizationParameters.from_arrays(scales, zps, precision, mode, strategy)
        if mode.case == "blockwise":
            return QuantizedTensorRecord(data, params, x.numel(), shape, bsc, bzp, bs)
        # Row-wise: the per-row scales ride in the parameters (the reference keeps no
        # block buffers for this mode); the device copies serve the kernels.
        return QuantizedTensorRecord(data, params, x.numel(), shape, bsc, bzp)

    def abi(self) -> mfa.QuantizedTensor:
        """The C-ABI view the quantised attention entry points take (tensor-wise or
        square-block-wise; the attention ABI has no per-row scale layout, and the reference
        itself applies only the first scale of a row-wise tensor, GEMMQuantization.swift:487)."""
        if self.parameters.mode.case == "rowWise":
            raise mfa.MFAError(2, "row-wise tensors have no attention operand layout")
        return mfa.quantized_tensor(self.data, self.parameters.precision, self.parameters.scale,
                                    self.parameters.zero_point, self.block_scales,
                                    self.block_zero_points, self.block_size_k or 0)

    # -- Codable
    def to_json_obj(self) -> dict:
        """encode(to:) (:953-985)."""
        header = {"version": SERIALIZATION_VERSION, "shape": [int(s) for s in self.original_shape]}
        if self.block_size_k is not None:
            header["blockSizeK"] = int(self.block_size_k)
        header.update({
            "quantMode": self.parameters.mode.to_json(),
            "dtype": PRECISION_NAME[P(self.parameters.precision)],
            "hasBlockScales": self.block_size_k is not None and self.block_scales is not None,
            "hasBlockZeroPoints": self.block_size_k is not None and self.block_zero_points is not None,
            "hasPrecomputedSums": self.precomputed_sums is not None,
            "elementCount": int(self.element_count),
        })
        out = {"header": header, "parameters": self.parameters.to_json(),
               "data": _b64(self.data)}
        if header["hasBlockScales"]:
            out["blockScales"] = _b64(self.block_scales)
        if header["hasBlockZeroPoints"]:
            out["blockZeroPoints"] = _b64(self.block_zero_points)
        if self.precomputed_sums is not None:
            out["precomputedSums"] = _b64(self.precomputed_sums)
        return out

    def encode(self) -> bytes:
        return json.dumps(self.to_json_obj()).encode()

    @staticmethod
    def from_json_obj(obj: dict, device="cuda:0") -> "QuantizedTensorRecord":
        """init(from:) (:987-1064) + decode(from:device:) (:1067-1076)."""
        import torch
        try:
            header = obj["header"]
            version = int(header["version"])
        except (KeyError, TypeError):
            raise FormatError("QuantizedTensor: missing header") from None
        if version != SERIALIZATION_VERSION:
            raise FormatError(f"Unsupported serialization version: {version}")
        params = QuantizationParameters.from_json(obj["parameters"])
        count = int(header["elementCount"])
        data = _unb64(obj["data"], torch.uint8, device)
        need = (count + 1) // 2 if P(params.precision) == P.INT4 else \
            count * {P.FP32: 4, P.FP16: 2, P.BF16: 2, P.INT8: 1}[P(params.precision)]
        if data.numel() < need:
            raise FormatError(f"data holds {data.numel()} bytes, {need} needed for {count} elements")
        bsk = header.get("blockSizeK")
        bsc = _unb64(obj["blockScales"], torch.float32, device) if header.get("hasBlockScales") else None
        bzp = (_unb64(obj["blockZeroPoints"], torch.int32, device)
               if header.get("hasBlockZeroPoints") else None)
        sums = (_unb64(obj["precomputedSums"], torch.uint8, device)
                if header.get("hasPrecomputedSums") else None)
        if params.mode.case == "rowWise" and bsc is None:
            bsc = torch.tensor(params.all_scales, dtype=torch.float32, device=device)
            bzp = torch.tensor(params.all_zero_points, dtype=torch.int32, device=device)
        return QuantizedTensorRecord(data, params, count, list(header["shape"]), bsc, bzp,
                                     None if bsk is None else int(bsk), sums)

    @staticmethod
    def decode(blob: bytes, device="cuda:0") -> "QuantizedTensorRecord":
        return QuantizedTensorRecord.from_json_obj(json.loads(blob), device)


def _b64(t) -> str:
    return base64.b64encode(t.detach().contiguous().view(-1).cpu().numpy().tobytes()).decode()


def _unb64(s: str, dtype, device):
    import numpy as np
    import torch
    raw = base64.b64decode(s)
    item = torch.empty((), dtype=dtype).element_size()
    if len(raw) % item:
        raise FormatError("buffer length is not a whole number of elements")
    arr = np.frombuffer(raw, dtype=np.uint8).copy()
    return torch.from_numpy(arr).view(dtype).to(device)


# ------------------------------------------------------------------- masking calibration
@dataclasses.dataclass
class MaskingCalibrationEntry:
    sequence_bucket: int
    head_dimension: int
    strategy: str              # MaskingStrategy raw value: "elementWise" | "bitmask"
    bitmask_ms: float
    element_wise_ms: float

    def to_json(self) -> dict:
        return {"bitmaskMs": float(self.bitmask_ms), "elementWiseMs": float(self.element_wise_ms),
                "headDimension": int(self.head_dimension),
                "sequenceBucket": int(self.sequence_bucket), "strategy": self.strategy}


@dataclasses.dataclass
class MaskingCalibration:
    """MaskingCalibration (MaskingStrategyHeuristic.swift:160-191)."""
    device_name: str
    entries: list

    def to_json(self) -> dict:
        return {"deviceName": self.device_name, "entries": [e.to_json() for e in self.entries]}

    @staticmethod
    def from_json(obj: dict) -> "MaskingCalibration":
        try:
            entries = []
            for e in obj["entries"]:
                if e["strategy"] not in ("elementWise", "bitmask"):
                    raise FormatError(f"unknown MaskingStrategy {e['strategy']!r}")
                entries.append(MaskingCalibrationEntry(int(e["sequenceBucket"]), int(e["headDimension"]),
                                                       e["strategy"], float(e["bitmaskMs"]),
                                                       float(e["elementWiseMs"])))
            return MaskingCalibration(str(obj["deviceName"]), entries)
        except KeyError as e:
            raise FormatError(f"MaskingCalibration: missing key {e}") from None


class MaskingCalibrationStore:
    """MaskingCalibrationStore (:415-447): prettyPrinted + sortedKeys JSON, atomic write."""

    @staticmethod
    def default_url(device_name: str, bundle_identifier: str = "FlashAttention") -> pathlib.Path:
        sanitized = device_name.replace(" ", "_")
        return (pathlib.Path.home() / ".cache" / bundle_identifier / "masking-calibration"
                / f"{sanitized}.json")

    @staticmethod
    def save(calibration: MaskingCalibration, path) -> None:
        path = pathlib.Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        # Swift's prettyPrinted style: two-space indent, "key" : value.
        text = json.dumps(calibration.to_json(), indent=2, sort_keys=True, separators=(",", " : "))
        tmp = path.with_name(path.name + ".tmp")
        tmp.write_text(text)
        os.replace(tmp, path)

    @staticmethod
    def load(path) -> MaskingCalibration:
        return MaskingCalibration.from_json(json.loads(pathlib.Path(path).read_text()))


class MaskingStrategyHeuristic:
    """MaskingStrategyHeuristic (:8-149): a process-wide cache keyed by (sequence bucket,
    head dimension) in front of defaultRule.  On gfx950 both strategies evaluate the same
    predicate per element, so the answer only labels the plan (results are identical)."""
    _lock = threading.Lock()
    _cache: dict = {}
    shared = None

    @staticmethod
    def sequence_bucket(sequence_length: int) -> int:
        return int(mfa.lib.mfa_masking_sequence_bucket(int(sequence_length)))

    def recommend(self, sequence_length: int, head_dimension: int) -> str:
        key = (self.sequence_bucket(sequence_length), int(head_dimension))
        with self._lock:
            hit = self._cache.get(key)
        if hit is not None:
            return hit
        rule = int(mfa.lib.mfa_masking_default_rule(int(sequence_length), int(head_dimension)))
        return "bitmask" if rule == 1 else "elementWise"

    def apply(self, calibration: MaskingCalibration) -> None:
        with self._lock:
            for e in calibration.entries:
                self._cache[(e.sequence_bucket, e.head_dimension)] = e.strategy

    def reset(self) -> None:
        with self._lock:
            self._cache.clear()


MaskingStrategyHeuristic.shared = MaskingStrategyHeuristic()
