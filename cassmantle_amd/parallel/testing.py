"""Fault-injecting worker generators for the supervised-group tests ("fault-injection
flags in the fake generator (fail / slow / NaN)").  A worker builds one through
``GroupSupervisor(gen_factory="cassmantle_amd.parallel.testing:stamped_generator")``; the fault is
configured through the worker environment:

* ``CASSMANTLE_FAULT_SLOT``: the device label (``cpu:1``, ``cuda:3``) whose worker misbehaves;
* ``CASSMANTLE_FAULT``: ``kill`` (the process exits mid-round, like an OOM kill or a driver
  crash), ``hang`` (the generation never returns but the process keeps heart-beating, like a
  wedged GPU kernel), ``fail`` (the generation raises), ``async_hang`` (``generate_device``
  returns at once, as the real pipeline does when it only QUEUES the work, but its completion
  event never fires: a GPU wedged inside the denoise graph), ``slow`` (every generation takes
  ``CASSMANTLE_FAULT_DELAY`` seconds longer: a straggler GPU), ``start_kill`` (the worker dies
  while its generator is being built: a fault during model load or graph capture), ``exit0``
  (the process leaves mid-round with exit code 0: no crash signature, still the culprit);
* ``CASSMANTLE_FAULT_TRIGGER``: a file; the fault fires only once it exists.  A ``{index}`` in
  the path is replaced by the slot's index, so a test can arm and disarm slots one by one
  (``CASSMANTLE_FAULT_SLOT`` may then name several slots, comma-separated);
* ``CASSMANTLE_FAULT_START_DELAY``: every worker sleeps this long while its generator is built
  (a slow model load / graph capture), fault or not.

Every image carries the generating slot's index in its top-left 8x8 block (value
``40 * (index + 1)``, robust to JPEG), so a test can tell which device drew a room's round.
"""
from __future__ import annotations

import os
import time

from ..game.content import ImageGenerationError, SolidImageGenerator


class StampedGenerator(SolidImageGenerator):
    def __init__(self, slot: str, res: int = 32) -> None:
        super().__init__(res)
        self.slot = slot
        self.index = _slot_index(slot)
        self.fault_mode = os.environ.get("CASSMANTLE_FAULT")
        self.trigger = _trigger(self.index)

    def _armed(self) -> bool:
        return _faulty(self.slot) and bool(self.trigger) and os.path.exists(self.trigger)

    def generate(self, prompts, negative_prompt, seeds):
        if self._armed():
            if self.fault_mode == "kill":
                os._exit(17)
            if self.fault_mode == "exit0":       # leaves mid-round with a CLEAN exit code
                os._exit(0)
            if self.fault_mode == "hang":
                time.sleep(3600)
            if self.fault_mode == "fail":
                raise ImageGenerationError("injected failure")
            if self.fault_mode == "slow":
                time.sleep(float(os.environ.get("CASSMANTLE_FAULT_DELAY", "1.0")))
        out = super().generate(prompts, negative_prompt, seeds)
        for im in out:
            im[:8, :8, :] = 40 * (self.index + 1)
        return out


class _Done:
    def query(self) -> bool:
        return True


class _Never:
    """A device event of work that never completes."""

    def query(self) -> bool:
        return False


class AsyncStampedGenerator(StampedGenerator):
    """``StampedGenerator`` with the device-resident interface of the SD pipeline
    (``generate_device`` -> ``DeviceImages``), host tensors standing in for HBM."""

    def generate_device(self, prompts, negative_prompt, seeds):
        import numpy as np
        import torch
        from ..pipeline import DeviceImages
        if self._armed() and self.fault_mode == "async_hang":
            img = torch.zeros((len(prompts), self.resolution, self.resolution, 3), dtype=torch.uint8)
            return DeviceImages(img, None, _Never())
        img = torch.from_numpy(np.stack(self.generate(prompts, negative_prompt, seeds)))
        return DeviceImages(img, None, _Done())


def _slot_index(slot: str) -> int:
    return int(slot.split(":")[1].split("#")[0]) if ":" in slot else 0


def _trigger(index: int) -> str:
    return os.environ.get("CASSMANTLE_FAULT_TRIGGER", "").replace("{index}", str(index))


def _faulty(slot: str) -> bool:
    return slot in os.environ.get("CASSMANTLE_FAULT_SLOT", "").split(",")


def stamped_generator(cfg, device: str, spec) -> StampedGenerator:
    slot = spec.slot or device
    trig = _trigger(_slot_index(slot))
    time.sleep(float(os.environ.get("CASSMANTLE_FAULT_START_DELAY", "0")))
    if os.environ.get("CASSMANTLE_FAULT") == "start_kill" and _faulty(slot) and trig and os.path.exists(trig):
        os._exit(17)                     # dies without reporting, before the "ready" message
    # CASSMANTLE_DEVICE_GEN=1: the device-resident interface without a fault (the ``ipc`` data
    # plane of the supervisor, host tensors standing in for HBM)
    dev_gen = os.environ.get("CASSMANTLE_FAULT") == "async_hang" or os.environ.get("CASSMANTLE_DEVICE_GEN") == "1"
    cls = AsyncStampedGenerator if dev_gen else StampedGenerator
    return cls(spec.slot or device, res=cfg.model.resolution)


def slot_of(img) -> int:
    """Inverse of the stamp: slot index that drew ``img`` (uint8 [H, W, 3])."""
    return int(round(float(img[:8, :8].mean()) / 40.0)) - 1
