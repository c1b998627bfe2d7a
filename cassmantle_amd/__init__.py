"""cassmantle_amd — MI355X-native prompt-guessing game server framework.

Layers: ``api`` (HTTP/WS contract) → ``game`` (rooms, rounds, sessions, scoring
rules, state store) → ``pipeline``/``scoring`` (on-device SD txt2img, batched GPU scorer) →
``models`` (CLIP, UNet, VAE, MiniLM on fused ops) → ``ops`` (hand-written HIP/CDNA4 kernels)
and ``parallel`` (room sharding over RCCL/xGMI, one process per GPU).
"""
__version__ = "0.1.0"
