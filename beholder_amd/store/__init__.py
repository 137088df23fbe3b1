"""Media stores (triton-core/db parity): memory, sqlite, postgres (wire-protocol client)."""
from .base import Media, MediaNotFound, MediaStore, StoreError, open_store  # noqa: F401
from .memory import MemoryStore  # noqa: F401
