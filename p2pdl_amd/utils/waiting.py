"""Drop-in for reference utils/waiting.py:4-21 (``wait_for_models``).

Contract kept: block until ``len(received_models) >= expected_count``,
polling once per ``poll`` seconds (reference :15 waits 1 s per poll), and
return True once the models are there.  One deliberate fix: the reference's
timeout can never fire (``threading.Event().wait(0)`` is False, so the
elapsed time it computes at :17 is always 0); here ``timeout`` seconds of
waiting return False, which the caller logs and proceeds on exactly as the
reference's caller intends (aggregator/aggregation.py:9-10).
"""
import logging
import time


def wait_for_models(received_models, expected_count, timeout=30, poll=1.0):
    start = time.monotonic()
    while len(received_models) < expected_count:
        if time.monotonic() - start > timeout:
            logging.warning("Timeout exceeded while waiting for model updates. Proceeding with aggregation.")
            return False
        time.sleep(poll)
    return True
