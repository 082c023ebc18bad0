from .manipulation import AsyncLoad, async_offload, async_reload, create_async_load  # noqa: F401
