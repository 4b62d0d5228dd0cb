"""Loader of the host-side staging extension (``csrc/staging_ext.cpp``, built in-tree by
``build.build_staging``). Loaded from its file without any build step at run time; ``None`` when
it is absent, and the plugin then stages updates in Python (same results, more host time)."""

from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import warnings
from types import ModuleType

import torch  # noqa: F401  (the extension links against torch's libraries)

from .build import STAGING_NAME, STAGING_PATH

_module: ModuleType | None = None
_tried = False


def module() -> ModuleType | None:
    global _module, _tried
    if not _tried:
        _tried = True
        if STAGING_PATH.exists() and os.environ.get("FEDAVG_PY_STAGING") != "1":
            try:
                loader = importlib.machinery.ExtensionFileLoader(STAGING_NAME, str(STAGING_PATH))
                spec = importlib.util.spec_from_file_location(STAGING_NAME, str(STAGING_PATH), loader=loader)
                assert spec is not None
                mod = importlib.util.module_from_spec(spec)
                loader.exec_module(mod)
                _module = mod
            except (ImportError, OSError) as e:  # e.g. built against another torch: stage in Python
                warnings.warn(f"staging extension {STAGING_PATH} not loadable ({e}); staging in Python",
                              RuntimeWarning, stacklevel=2)
    return _module
