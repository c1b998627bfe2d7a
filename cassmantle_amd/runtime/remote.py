"""Remote generation over HTTP (reference parity path; off by default — the box has no network).

The reference generates all content through Hugging Face inference endpoints:
``api_call`` (``src/utils.py:32-72``) retries up to ``max_retries`` times, sleeping
``10·(retry+1)`` s when the response status is in ``{503}`` (model loading), aborts on any other
error and returns the raw body bytes or ``None``; the session uses a 60 s total timeout and
``raise_for_status=True`` (``src/backend.py:98-101``).  ``generate_prompt`` posts
``{"inputs": seed, "parameters": {"min_new_tokens": 32, "max_new_tokens": 96}}`` and keeps two
sentences of ``generated_text[len(seed):]`` (``src/backend.py:240-268``); ``generate_image``
posts the styled prompt with the negative prompt and decodes the image bytes
(``src/backend.py:270-295``).

These adapters plug into the same synchronous generator interfaces the on-device paths use
(the game layer calls generators from worker threads), so a deployment can mix e.g. remote
prompts with on-device images.  The retry unit is configurable (``ModelConfig.remote_retry_s``)
so tests run in milliseconds.
"""
from __future__ import annotations

import asyncio
import io
import json
import logging
from typing import Any, Dict, Optional, Set

import numpy as np

from ..game.content import ImageGenerationError, ImageGenerator
from ..game.prompts import PromptGenerator, postprocess_generation

log = logging.getLogger("cassmantle.remote")


async def api_call(session, method: str, url: str, headers: Optional[Dict[str, str]] = None,
                   json_payload: Optional[Dict[str, Any]] = None, max_retries: int = 5,
                   retry_on_status_codes: Optional[Set[int]] = None, retry_unit_s: float = 10.0,
                   ssl: bool = False) -> Optional[bytes]:
    """Body bytes, or ``None`` after ``max_retries`` retryable statuses / any other error."""
    import aiohttp
    retry_on = retry_on_status_codes or {503}
    for retry in range(max_retries):
        try:
            async with session.request(method, url, headers=headers, json=json_payload, ssl=ssl) as resp:
                return await resp.read()
        except aiohttp.ClientResponseError as e:
            if e.status in retry_on:
                log.info("retry %d/%d: status %d from %s", retry + 1, max_retries, e.status, url)
                await asyncio.sleep((retry + 1) * retry_unit_s)
                continue
            log.warning("HTTP error: %s", e)
            break
        except Exception as e:  # noqa: BLE001 - reference aborts on any other error
            log.warning("request error: %s", e)
            break
    log.warning("max retries reached or an error occurred (%s)", url)
    return None


class _RemoteBase:
    def __init__(self, url: str, token: Optional[str] = None, timeout_s: float = 60.0,
                 max_retries: int = 5, retry_unit_s: float = 10.0) -> None:
        self.url = url
        self.headers = {"Authorization": f"Bearer {token}"} if token else {}
        self.timeout_s = timeout_s
        self.max_retries = max_retries
        self.retry_unit_s = retry_unit_s

    async def _post(self, payload: Dict[str, Any]) -> Optional[bytes]:
        import aiohttp
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout_s),
                                         raise_for_status=True) as s:
            return await api_call(s, "POST", self.url, headers=self.headers, json_payload=payload,
                                  max_retries=self.max_retries, retry_on_status_codes={503},
                                  retry_unit_s=self.retry_unit_s)

    def post(self, payload: Dict[str, Any]) -> Optional[bytes]:
        # generators are called from worker threads (asyncio.to_thread): own event loop here
        return asyncio.run(self._post(payload))


class RemotePromptGenerator(_RemoteBase, PromptGenerator):
    def __init__(self, url: str, min_new_tokens: int = 32, max_new_tokens: int = 96, **kw) -> None:
        super().__init__(url, **kw)
        self.min_new_tokens, self.max_new_tokens = min_new_tokens, max_new_tokens

    def generate(self, seed: str, is_seed: bool) -> Optional[str]:
        body = self.post({"inputs": seed, "parameters": {"min_new_tokens": self.min_new_tokens,
                                                         "max_new_tokens": self.max_new_tokens}})
        if body is None:
            return None
        try:
            text = json.loads(body)[0].get("generated_text", "")
        except (ValueError, IndexError, KeyError, AttributeError, TypeError):
            return None
        return postprocess_generation(text, seed, echoed=True)


class RemoteImageGenerator(_RemoteBase, ImageGenerator):
    def __init__(self, url: str, resolution: int = 1024, **kw) -> None:
        super().__init__(url, **kw)
        self.resolution = resolution

    def generate(self, prompts, negative_prompt, seeds):
        from PIL import Image
        out = []
        for p in prompts:
            body = self.post({"inputs": p, "parameters": {"negative_prompt": negative_prompt}})
            if body is None:
                raise ImageGenerationError("remote image generation failed")
            try:
                img = Image.open(io.BytesIO(body)).convert("RGB")
            except Exception as e:  # noqa: BLE001
                raise ImageGenerationError(f"undecodable image: {e}") from e
            out.append(np.asarray(img, dtype=np.uint8))
        return out
