"""`python sheeprl.py exp=<preset> ...` (reference: sheeprl.py)."""
from sheeprl_prey_amd.cli import run

if __name__ == "__main__":
    run()
