#!/usr/bin/env python3
"""`python server.py [server_ip]` — start the coordinator (reference CLI form)."""
import sys

from distributedvolunteercomputing_amd.cli.main import server_main

if __name__ == "__main__":
    sys.exit(server_main())
