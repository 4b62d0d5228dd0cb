"""Plugin registry: algorithm name -> (client, server, endpoints, algorithm factory).

Same API as the reference's ``AlgorithmRepository``
(``simulation_lib/algorithm_repository.py:5-68``). ``create_server`` instantiates
``algorithm_cls()`` and hands it to the server as ``algorithm=`` (:62-66); registering the
HIP ``FedAVGAlgorithm`` under ``"fed_avg"`` is the drop-in point (the reference's built-in
registration is ``common_method/__init__.py:6-11``).
"""

from __future__ import annotations

from collections.abc import Callable
from typing import Any


class AlgorithmRepository:
    config: dict[str, dict] = {}

    @classmethod
    def register_algorithm(
        cls,
        algorithm_name: str,
        client_cls: Callable[..., Any],
        server_cls: Callable[..., Any],
        client_endpoint_cls: Callable[..., Any] | None = None,
        server_endpoint_cls: Callable[..., Any] | None = None,
        algorithm_cls: Callable[[], Any] | None = None,
    ) -> None:
        assert algorithm_name not in cls.config
        entry: dict[str, Any] = {"client_cls": client_cls, "server_cls": server_cls}
        optional = {
            "client_endpoint_cls": client_endpoint_cls,
            "server_endpoint_cls": server_endpoint_cls,
            "algorithm_cls": algorithm_cls,
        }
        entry.update({k: v for k, v in optional.items() if v is not None})
        cls.config[algorithm_name] = entry

    @classmethod
    def has_algorithm(cls, algorithm_name: str) -> bool:
        return algorithm_name in cls.config

    @classmethod
    def create_client(
        cls, algorithm_name: str, kwargs: dict, endpoint_kwargs: dict, **extra_kwargs: Any
    ) -> Any:
        entry = cls.config[algorithm_name]
        if "client_endpoint_cls" in entry:
            endpoint_kwargs["endpoint_cls"] = entry["client_endpoint_cls"]
        endpoint = extra_kwargs["context"].create_client_endpoint(**endpoint_kwargs)
        return entry["client_cls"](endpoint=endpoint, **kwargs, **extra_kwargs)

    @classmethod
    def create_server(
        cls, algorithm_name: str, kwargs: dict, endpoint_kwargs: dict, **extra_kwargs: Any
    ) -> Any:
        entry = cls.config[algorithm_name]
        if "server_endpoint_cls" in entry:
            endpoint_kwargs["endpoint_cls"] = entry["server_endpoint_cls"]
        endpoint = extra_kwargs["context"].create_server_endpoint(**endpoint_kwargs)
        if "algorithm_cls" in entry:
            assert "algorithm" not in extra_kwargs
            extra_kwargs["algorithm"] = entry["algorithm_cls"]()
        return entry["server_cls"](endpoint=endpoint, **kwargs, **extra_kwargs)
