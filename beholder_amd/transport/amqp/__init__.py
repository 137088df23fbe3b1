"""AMQP 0-9-1 transport: wire codec, asyncio client, consumer source, publisher, test broker."""
from .wire import AmqpError, parse_url  # noqa: F401
from .connection import Channel, Connection, connect  # noqa: F401
from .source import AmqpPublisher, AmqpSource, publish_frames  # noqa: F401
from .broker import AmqpBroker  # noqa: F401
