"""MI355X-native model-update compression for COALA (the package the reference leaves empty:
/root/reference/coala/compression/__init__.py is 0 bytes).

Public surface:
  CompressionClientMixin / CompressionServerMixin — hook mixins (plugin.py)
  UpdateCodec, CompressedUpdate                    — state_dict codec + picklable carrier (codec.py)
  CompressedModel, compress_model                  — download direction: compressed global model (download.py)
  CodecPlan, Encoded                               — batched device-level API over the C ABI (plan.py)
  k_for, SegmentTable                              — CodecSpec v1 host logic (spec.py)
"""
from . import wire
from .codec import CompressedUpdate, FlatState, HipBackend, UpdateCodec, flatten_state, module_with_state
from .download import CompressedModel, compress_model, skeleton_of
from .pipeline import SplitPipeline, split_lanes
from .plan import CodecPlan, Encoded
from .plugin import CompressionClientMixin, CompressionServerMixin
from .spec import ALIGN, RAW_BITS, SegmentTable, SubTable, k_for

__all__ = ["wire", "SplitPipeline", "CompressedModel", "compress_model", "skeleton_of", "split_lanes", "SubTable", "CompressedUpdate", "FlatState", "HipBackend", "UpdateCodec", "flatten_state", "module_with_state",
           "CodecPlan", "Encoded", "CompressionClientMixin", "CompressionServerMixin", "ALIGN", "RAW_BITS",
           "SegmentTable", "k_for"]
