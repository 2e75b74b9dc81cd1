"""mjpy: import-compatible stand-in for the reference's rl/env/mjpy package
(`from mjpy.bind import MjClass, EventTrack`, MjEnv.py:18) over the MI355X C ABI."""
