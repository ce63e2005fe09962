"""Timing probe (wrong outputs): Philox rounds per spawn evaluation, 10 (shipped) vs 7 vs 1,
to size the Philox share of the C5 step kernel."""
_OLD = "    for (int r = 0; r < 10; r++) {\n        const uint64_t p0"
VARIANTS = {
    "ph10": [],
    "ph7": [("sl_device.h", _OLD, _OLD.replace("r < 10", "r < 7"))],
    "ph1": [("sl_device.h", _OLD, _OLD.replace("r < 10", "r < 1"))],
}
