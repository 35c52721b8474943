"""CPU: the host slot device selection (include/s3dlio_gpu.h, host-buffer
drop-ins) as a pure function of the env values and the device count."""
import pytest

from s3dlio_amd.device import parse_devices


def test_default_every_visible_gpu():
    assert parse_devices(None, None, 8) == list(range(8))
    assert parse_devices("", "", 1) == [0]


def test_pin_one_device():
    assert parse_devices("3", None, 8) == [3]
    assert parse_devices("3", "0,1", 8) == [3]          # the pin wins over the list
    assert parse_devices(" 0 ", None, 1) == [0]


def test_device_list_with_repeats():
    assert parse_devices(None, "0,1,1,7", 8) == [0, 1, 1, 7]
    assert parse_devices(None, "0,0,0", 1) == [0, 0, 0]


@pytest.mark.parametrize("pin,lst,ndev", [("8", None, 8), ("x", None, 2), ("-1", None, 2), (None, "0,9", 8),
                                          (None, "0,,1", 8), (None, "0,1,", 8), (None, "a", 8), (None, None, 0)])
def test_bad_values_raise(pin, lst, ndev):
    with pytest.raises(ValueError):
        parse_devices(pin, lst, ndev)


def test_rank_of_a_multi_process_job_keeps_to_its_gpu():
    """under torch.distributed.run every rank sees every GPU; with
    neither env var its host slots stay on LOCAL_RANK's GPU."""
    assert parse_devices(None, None, 8, "3", "8") == [3]
    assert parse_devices(None, None, 1, "5", "8") == [0]            # one visible GPU per rank
    assert parse_devices(None, None, 8, "3", "1") == list(range(8))  # a single-process job
    assert parse_devices(None, None, 8, None, "8") == list(range(8))
    assert parse_devices(None, None, 8, "x", "8") == list(range(8))  # unparsable: the default
    assert parse_devices("6", None, 8, "3", "8") == [6]              # explicit settings win
    assert parse_devices(None, "0,1", 8, "3", "8") == [0, 1]


def test_abi_wrapper_matches_env_form():
    from s3dlio_amd._lib import lib
    import ctypes
    out = (ctypes.c_int * 8)()
    n = ctypes.c_int()
    assert lib.s3dg_host_parse_devices(None, None, 4, out, 8, ctypes.byref(n)) == 0
    assert list(out[:n.value]) == [0, 1, 2, 3]
