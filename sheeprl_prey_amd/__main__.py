from sheeprl_prey_amd.cli import run

if __name__ == "__main__":
    run()
