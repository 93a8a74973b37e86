"""MI355X-native (gfx950) OCTO-style multimodal transformer training path with token merging.

Mirrors the module/config API of the reference ``multi_modal_transformers`` package
(tokenizers -> attention_blocks -> action_heads, models.octo) on PyTorch-ROCm; every hot op runs
in the hand-written HIP library ``libmmt_hip.so`` (C ABI: include/mmt_api.h).
"""
__version__ = "0.1.0"
