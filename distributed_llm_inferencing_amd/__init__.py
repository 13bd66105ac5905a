"""distributed_llm_inferencing_amd — an MI355X-native (gfx950 / CDNA4) master/worker sharded
LLM inference hub with the capabilities and HTTP API of MihirPanpatil/Distributed-LLM-Inferencing.

Layers (see README.md / SURVEY.md §7):
    control/   Flask master: node registry, request queue, dispatcher, dashboard (API-compatible)
    worker/    per-GPU Flask worker with the reference's /health /load_model /load_shard ...
    engine/    continuous-batching scheduler, paged KV cache, hipGraph decode runner
    models/    Llama-3 / Mixtral / GPT-2 on our ops, random-init or safetensors weights
    ops/       hand-written HIP kernels for gfx950 (csrc/kernels) + PyTorch references
    parallel/  pipeline (RCCL send/recv over xGMI), expert-parallel all-to-all, launcher
    shard/     layer-contiguous HBM-aware shard planner/writer (metadata.json compatible)
    runtime/   C++ host runtime: KV block allocator, safetensors -> hipMemcpyAsync loader
"""
__version__ = "0.1.0"
