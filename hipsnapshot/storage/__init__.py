"""Storage plugins: fs (native engine), s3, gcs, memory, and the URL registry."""

from .registry import (  # noqa: F401
    register_storage_plugin,
    split_url,
    url_to_storage_plugin,
    url_to_storage_plugin_in_event_loop,
)
