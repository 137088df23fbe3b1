"""Media table layout: table name + one column per :class:`~.base.Media` field.

``triton-core/db``'s migrations are not vendored (index.js:42 ``new Storage()``; reads at
index.js:76,140, the status write at index.js:68), so the column names are a documented guess
(snake_case). ``service.store.table`` and ``service.store.columns`` override it::

    service:
      store:
        table: public.media
        columns: {creatorId: "creatorId", metadataId: "metadataId"}   # the rest keep defaults

Identifiers are validated (``[A-Za-z_][A-Za-z0-9_]*``, optionally ``schema.table``) and emitted
double-quoted, so a camelCase column created by an ORM matches exactly (unquoted Postgres
identifiers fold to lower case). The SELECT always lists the columns in ``Media`` field order,
so a row maps positionally onto ``Media`` whatever the names are (the compiled handlers rely on
that: they run the store's ``_select`` text and build the Media from the row positions).
"""
from __future__ import annotations

import re
from typing import Dict, Mapping, Optional, Tuple

from .base import FIELDS

#: our default guess: snake_case of the api.Media field names
DEFAULT_COLUMNS: Dict[str, str] = {
    "id": "id", "name": "name", "creator": "creator", "creatorId": "creator_id", "type": "type",
    "source": "source", "sourceURI": "source_uri", "metadata": "metadata", "metadataId": "metadata_id",
    "status": "status",
}
_TEXT = frozenset(("id", "name", "creatorId", "sourceURI", "metadataId"))
_IDENT = re.compile(r"^[A-Za-z_][A-Za-z0-9_]*$")


def _quote(ident: str) -> str:
    if not _IDENT.match(ident):
        raise ValueError(f"invalid SQL identifier {ident!r}")
    return f'"{ident}"'


class MediaSchema:
    """Table + column mapping, and the SQL text of the store's statements for it.

    ``ph`` builds the placeholder of the i-th (1-based) parameter: ``$i`` for Postgres,
    ``?`` for SQLite.
    """

    def __init__(self, table: str = "media", columns: Optional[Mapping[str, str]] = None):
        cols = dict(DEFAULT_COLUMNS)
        for k, v in (columns or {}).items():
            if k not in DEFAULT_COLUMNS:
                raise ValueError(f"unknown media field {k!r} in store columns (fields: {', '.join(FIELDS)})")
            cols[k] = str(v)
        parts = table.split(".")
        if not 1 <= len(parts) <= 2:
            raise ValueError(f"invalid table name {table!r}")
        self.table = table
        self.columns = cols
        self.qtable = ".".join(_quote(p) for p in parts)
        self.qcols: Tuple[str, ...] = tuple(_quote(cols[f]) for f in FIELDS)
        if len(set(cols[f] for f in FIELDS)) != len(FIELDS):
            raise ValueError("store columns must be distinct")

    @property
    def is_default(self) -> bool:
        return self.table == "media" and self.columns == DEFAULT_COLUMNS

    def col(self, field: str) -> str:
        return self.qcols[FIELDS.index(field)]

    def select_by_id(self, ph) -> str:
        return f"SELECT {', '.join(self.qcols)} FROM {self.qtable} WHERE {self.col('id')} = {ph(1)}"

    def update_status(self, ph) -> str:
        return f"UPDATE {self.qtable} SET {self.col('status')} = {ph(1)} WHERE {self.col('id')} = {ph(2)}"

    def upsert(self, ph, excluded: str = "EXCLUDED") -> str:
        vals = ",".join(ph(i + 1) for i in range(len(FIELDS)))
        sets = ", ".join(f"{c} = {excluded}.{c}" for c in self.qcols[1:])
        return (f"INSERT INTO {self.qtable} ({', '.join(self.qcols)}) VALUES ({vals}) "
                f"ON CONFLICT ({self.col('id')}) DO UPDATE SET {sets}")

    def count(self) -> str:
        return f"SELECT COUNT(*) FROM {self.qtable}"

    def create_table(self, int_type: str = "INTEGER") -> str:
        defs = []
        for f, c in zip(FIELDS, self.qcols):
            if f == "id":
                defs.append(f"{c} TEXT PRIMARY KEY")
            elif f in _TEXT:
                defs.append(f"{c} TEXT NOT NULL DEFAULT ''")
            else:
                defs.append(f"{c} {int_type} NOT NULL DEFAULT 0")
        return f"CREATE TABLE IF NOT EXISTS {self.qtable} ({', '.join(defs)})"

    def describe(self) -> str:
        """One line for the startup log: the table and every field -> column."""
        return f"table={self.table} columns=" + ",".join(f"{f}:{self.columns[f]}" for f in FIELDS)


def pg_ph(i: int) -> str:
    return f"${i}"


def sqlite_ph(i: int) -> str:
    return "?"


def text_field_indexes() -> Tuple[int, ...]:
    return tuple(i for i, f in enumerate(FIELDS) if f in _TEXT)
