#!/usr/bin/env python3
"""`python worker.py [server_ip own_ip]` — start a volunteer client (reference CLI form)."""
import sys

from distributedvolunteercomputing_amd.cli.main import worker_main

if __name__ == "__main__":
    sys.exit(worker_main())
