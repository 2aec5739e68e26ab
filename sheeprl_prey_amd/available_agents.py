"""Print the registered algorithms (reference: ``sheeprl/available_agents.py``)."""
from sheeprl_prey_amd.utils.registry import tasks


def available_agents() -> None:
    import sheeprl_prey_amd  # noqa: F401

    try:
        from rich.console import Console
        from rich.table import Table

        table = Table(title="SheepRL-prey (MI355X) Agents")
        table.add_column("Module")
        table.add_column("Algorithm")
        table.add_column("Entrypoint")
        table.add_column("Decoupled")
        for module, impls in tasks.items():
            for impl in impls:
                table.add_row(module, impl["name"], impl["entrypoint"], str(impl["decoupled"]))
        Console().print(table)
    except ImportError:  # pragma: no cover
        for module, impls in tasks.items():
            for impl in impls:
                print(module, impl["name"], impl["entrypoint"], impl["decoupled"])


if __name__ == "__main__":
    available_agents()
