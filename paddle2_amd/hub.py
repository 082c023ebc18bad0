"""paddle.hub (reference: python/paddle/hapi/hub.py:185 list, :235 help, :283 load).

A hub repo is a directory with a ``hubconf.py`` whose public callables are model entry points and
whose optional ``dependencies`` list names required modules.  ``source='local'`` loads from a path;
'github'/'gitee' resolve to the reference's cache layout (``~/.cache/paddle/hub/<owner>_<repo>_<branch>``)
and need that cache to exist, since there is no network access.
"""
from __future__ import annotations

import builtins
import importlib.util
import os
import sys

_HUBCONF = "hubconf.py"
_SOURCES = ("github", "gitee", "local")


def _hub_dir():
    return os.path.join(os.path.expanduser(os.environ.get("HUB_HOME", "~/.cache/paddle/hub")))


def _repo_dir(repo_dir, source, force_reload):
    if source not in _SOURCES:
        raise ValueError(f'Unknown source: "{source}". Allowed values: "github" | "gitee" | "local".')
    if source == "local":
        return repo_dir
    owner_repo, _, branch = repo_dir.partition(":")
    branch = branch or ("main" if source == "github" else "master")
    owner, _, name = owner_repo.partition("/")
    cached = os.path.join(_hub_dir(), f"{owner}_{name}_{branch}")
    if force_reload or not os.path.isdir(cached):
        raise RuntimeError(f"hub repo {repo_dir!r} is not cached at {cached} and cannot be downloaded offline")
    return cached


def _import_hubconf(repo_dir):
    path = os.path.join(repo_dir, _HUBCONF)
    if not os.path.exists(path):
        raise FileNotFoundError(f"no {_HUBCONF} in {repo_dir}")
    spec = importlib.util.spec_from_file_location("hubconf", path)
    mod = importlib.util.module_from_spec(spec)
    sys.path.insert(0, repo_dir)
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.path.remove(repo_dir)
    missing = [d for d in getattr(mod, "dependencies", []) if importlib.util.find_spec(d) is None]
    if missing:
        raise RuntimeError(f"missing dependencies: {', '.join(missing)}")
    return mod


def _entry(mod, name):
    fn = getattr(mod, name, None)
    if fn is None or not callable(fn):
        raise RuntimeError(f"Cannot find callable {name} in hubconf")
    return fn


def list(repo_dir, source="github", force_reload=False):  # noqa: A001
    mod = _import_hubconf(_repo_dir(repo_dir, source, force_reload))
    return [k for k in dir(mod) if callable(getattr(mod, k)) and not k.startswith("_")
            and not isinstance(getattr(mod, k), type(builtins))]


def help(repo_dir, model, source="github", force_reload=False):  # noqa: A001
    return _entry(_import_hubconf(_repo_dir(repo_dir, source, force_reload)), model).__doc__


def load(repo_dir, model, source="github", force_reload=False, **kwargs):
    return _entry(_import_hubconf(_repo_dir(repo_dir, source, force_reload)), model)(**kwargs)
