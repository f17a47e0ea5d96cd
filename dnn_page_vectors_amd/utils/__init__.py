"""Small utilities: filesystem helpers, logging, metrics and tracing."""
