"""Kernel-side cross-stream signal (pcst_signal_write / pcst_signal_wait, _hip.DeviceSignal): the
sampling loop's loop -> side dependency.  Work enqueued after a wait must see everything the
producer stream wrote before the matching signal, under load and across many rounds."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_signal_orders_consumer_after_producer():
    from pointcloud_style_transfer_amd import _hip

    dev = torch.device("cuda", 0)
    prod = torch.cuda.Stream(device=dev, priority=-1)
    cons = torch.cuda.Stream(device=dev)
    sig = _hip.DeviceSignal(dev)
    a = torch.randn(2048, 2048, device=dev)
    buf = torch.zeros(2048, 2048, device=dev)
    outs = []
    for r in range(20):
        prod.wait_stream(torch.cuda.current_stream())
        prod.wait_stream(cons)  # the previous round's copy has read buf
        with torch.cuda.stream(prod):
            # a long producer chain ending in the value the consumer must see
            y = a
            for _ in range(4):
                y = torch.tanh(y @ a) * 0.5
            buf.copy_(y + float(r))
            sig.signal(prod)
        sig.wait(cons)
        with torch.cuda.stream(cons):
            outs.append((buf.clone(), r))
        buf.record_stream(cons)
    torch.cuda.synchronize()
    assert not sig.timed_out()
    y = a
    for _ in range(4):
        y = torch.tanh(y @ a) * 0.5
    for got, r in outs:
        torch.testing.assert_close(got, y + float(r), rtol=0, atol=0)


def test_signal_values_are_monotonic_per_flag():
    from pointcloud_style_transfer_amd import _hip

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    sig = _hip.DeviceSignal(dev)
    for _ in range(5):
        sig.signal(s)
        sig.wait(s)  # the same stream: already satisfied when it runs
    torch.cuda.synchronize()
    assert int(sig.flag[0].item()) == 5 and sig.value == 5 and not sig.timed_out()
