"""Side-effect sinks (L2 of SURVEY.md §1): Trello, Telegram, Emby over a pluggable HTTP client."""
from .http import (AiohttpClient, HttpClient, HttpError, HttpResponse, RecordingHttpClient,  # noqa: F401
                   SinkObserver, encode_query, observed, parse_query, redact, with_query)
from .h1 import H1Client  # noqa: F401
from .trello import COMMENT_FALLBACK, TrelloClient  # noqa: F401
from .telegram import TelegramClient, deployed_text  # noqa: F401
from .emby import EmbyClient  # noqa: F401
