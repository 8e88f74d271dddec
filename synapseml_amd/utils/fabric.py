"""Fabric / token helpers (reference: core/.../fabric/{FabricClient, TokenLibrary, OpenAITokenLibrary}.scala).

Hosted token services are not reachable offline; tokens come from the environment
(``SYNAPSEML_AAD_TOKEN`` / ``SYNAPSEML_OPENAI_TOKEN``) and the ML workload endpoint from
``SYNAPSEML_FABRIC_ENDPOINT``. Cognitive-service transformers use these as their default auth when
``running_on_fabric()``."""
from __future__ import annotations

import os
from typing import Optional

from .platform import running_on_fabric


class TokenLibrary:
    @staticmethod
    def getAccessToken(audience: str = "ml") -> Optional[str]:  # noqa: N802
        return os.environ.get("SYNAPSEML_AAD_TOKEN")

    @staticmethod
    def getAuthHeader() -> Optional[str]:  # noqa: N802
        tok = TokenLibrary.getAccessToken()
        return None if tok is None else "Bearer " + tok


class OpenAITokenLibrary(TokenLibrary):
    @staticmethod
    def getAccessToken(audience: str = "openai") -> Optional[str]:  # noqa: N802
        return os.environ.get("SYNAPSEML_OPENAI_TOKEN") or os.environ.get("SYNAPSEML_AAD_TOKEN")


class FabricClient:
    @staticmethod
    def MLWorkloadEndpointML() -> Optional[str]:  # noqa: N802
        return os.environ.get("SYNAPSEML_FABRIC_ENDPOINT")

    @staticmethod
    def available() -> bool:
        return running_on_fabric() and FabricClient.MLWorkloadEndpointML() is not None


__all__ = ["TokenLibrary", "OpenAITokenLibrary", "FabricClient"]
