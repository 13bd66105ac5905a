"""Cross-cutting utilities: tracing (roctx, request spans), fault injection, logging."""
