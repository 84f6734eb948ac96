"""CLI entry points: the status command against a live coordinator, the config listing, the
server CLI's data-plane flag."""
import json

from distributedvolunteercomputing_amd.cli import main as cli
from distributedvolunteercomputing_amd.control.coordinator import coordinator


def test_status_command(capsys):
    c = coordinator("127.0.0.1", 0, ephemeral_ports=True, data_plane="p2p")
    try:
        assert cli.main(["status", "127.0.0.1", "--port", str(c.control_port)]) == 0
        st = json.loads(capsys.readouterr().out)
        assert st["data_plane"] == "p2p" and st["workers"] == [] and "peers" in st
    finally:
        c.exit_threads()


def test_config_listing_and_usage(capsys):
    assert cli.main(["status", "--config"]) == 0
    assert "VCX_GEMM" in capsys.readouterr().out
    assert cli.main([]) == 2
    assert "status" in capsys.readouterr().out
