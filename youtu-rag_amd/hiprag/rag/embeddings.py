"""Embedders behind BaseEmbedder, and the factory that picks one.

* ServiceEmbedder -- client of the reference's remote embedding service, same
  wire format and batching (utu/rag/embeddings/service_embedder.py:16-177):
  POST {url}/embed_docs {"docs": [...]} / {url}/embed_query {"query": q}, reply
  {"embedding": base64(fp32 bytes), "shape": [...]}; texts are sent in
  sequential batches of ``batch_size``; GET {url}/model_id health check raising
  ConnectionError / TimeoutError (:44-61); transient 502/503/timeouts retried
  (utu/rag/utils/http_retry.py:16-60).
* TorchRocmEmbedder (hiprag.rag.rocm_embedder) -- the in-process PyTorch-ROCm
  replacement for that remote hop (provider "rocm"/"huggingface"/"local").
* EmbedderFactory.create(backend, **kwargs) / create_embedder -- as
  utu/rag/embeddings/factory.py:14-160 ("auto" reads UTU_EMBEDDING_URL).
"""
from __future__ import annotations

import base64
import logging
import os
import time

import numpy as np

from .base import BaseEmbedder

logger = logging.getLogger(__name__)


def decode_embedding_payload(payload: dict) -> list:
    """{"embedding": b64 fp32, "shape": [...]} -> nested lists (service_embedder.py:115-118)."""
    raw = base64.b64decode(payload["embedding"].encode("ascii"))
    return np.frombuffer(raw, dtype=np.float32).reshape(payload["shape"]).tolist()


def post_with_retry(url: str, json_data: dict, timeout: float = 60, max_retries: int = 3,
                    retry_delay: float = 2.0) -> dict:
    """POST returning JSON; retries 502/503, timeouts and connection errors."""
    import requests

    last: Exception | None = None
    for attempt in range(max_retries):
        try:
            rsp = requests.post(url, json=json_data, timeout=timeout)
            if rsp.status_code in (502, 503):
                last = requests.exceptions.HTTPError(f"{rsp.status_code} from {url}")
            else:
                rsp.raise_for_status()
                return rsp.json()
        except (requests.exceptions.Timeout, requests.exceptions.ConnectionError) as e:
            last = e
        if attempt + 1 < max_retries:
            time.sleep(retry_delay)
    raise RuntimeError(f"request to {url} failed after {max_retries} attempts: {last}")


class ServiceEmbedder(BaseEmbedder):
    def __init__(self, service_url: str, batch_size: int = 64, max_retries: int = 3, retry_delay: float = 2.0,
                 check_health: bool = True):
        self.service_url = service_url.rstrip("/")
        self.batch_size = int(batch_size)
        self.max_retries = max_retries
        self.retry_delay = retry_delay
        if self.batch_size < 1:
            raise ValueError("batch_size must be at least one")
        if check_health:
            self._check_service_health()

    def _check_service_health(self):
        import requests

        try:
            rsp = requests.get(f"{self.service_url}/model_id", timeout=5)
            rsp.raise_for_status()
            logger.info("embedding service healthy, model id %s", rsp.json())
        except requests.exceptions.ConnectionError as e:
            raise ConnectionError(f"Embedding service unreachable: {self.service_url}") from e
        except requests.exceptions.Timeout as e:
            raise TimeoutError(f"Embedding service timeout: {self.service_url}") from e

    def _post(self, route: str, body: dict, timeout: float) -> dict:
        return post_with_retry(f"{self.service_url}/{route}", body, timeout=timeout, max_retries=self.max_retries,
                               retry_delay=self.retry_delay)

    async def embed_texts(self, texts: list[str]) -> list[list[float]]:
        out: list[list[float]] = []
        for i in range(0, len(texts), self.batch_size):
            batch = list(texts[i:i + self.batch_size])
            out.extend(decode_embedding_payload(self._post("embed_docs", {"docs": batch}, 60)))
        return out

    async def embed_query(self, query: str) -> list[float]:
        return decode_embedding_payload(self._post("embed_query", {"query": query}, 30))


class EmbedderFactory:
    @staticmethod
    def create(backend: str = "auto", **kwargs) -> BaseEmbedder:
        if backend == "auto":
            url = os.getenv("UTU_EMBEDDING_URL")
            if not url:
                raise ValueError("Could not auto-detect embedder configuration. "
                                 "Please set UTU_EMBEDDING_URL environment variable.")
            return EmbedderFactory._openai(base_url=url, **kwargs)
        if backend == "service":
            kwargs.pop("batch_delay", None)
            url = kwargs.pop("service_url", None) or os.getenv("UTU_EMBEDDING_URL")
            if not url:
                raise ValueError("service_url is required for service embedder")
            return ServiceEmbedder(service_url=url, **kwargs)
        if backend == "openai":
            return EmbedderFactory._openai(**kwargs)
        if backend in ("rocm", "huggingface", "local"):
            from .rocm_embedder import TorchRocmEmbedder

            return TorchRocmEmbedder(**kwargs)
        raise ValueError(f"Unknown embedder backend: {backend}. Supported backends: auto, openai, service, rocm")

    @staticmethod
    def _openai(**kwargs) -> BaseEmbedder:
        try:
            import openai  # noqa: F401
        except ImportError as e:
            raise ImportError("the OpenAI-compatible embedder needs the `openai` package; use backend='rocm' for "
                              "the in-process MI355X embedder or 'service' for the HTTP service") from e
        raise NotImplementedError("OpenAI-compatible remote embedder is outside the hiprag hot path")


def create_embedder(backend: str = "auto", **kwargs) -> BaseEmbedder:
    return EmbedderFactory.create(backend, **kwargs)
