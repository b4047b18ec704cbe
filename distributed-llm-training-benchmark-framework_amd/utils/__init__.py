"""dltb.utils — distributed setup, timers, memory and platform helpers."""
