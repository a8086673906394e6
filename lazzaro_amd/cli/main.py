"""Interactive CLI (reference ``src/lazzaro/cli/main.py:5-153``).

Same commands: /quit /start /end /stats /profile /memories [n] /consolidate
/merge /prune [t] /config /set k v /save [f] /load [f] /help; plain text goes
to ``chat_stream``. Differences: works offline (local LLM + hash/on-device
embedder when no OPENAI_API_KEY), /save and /load work (the reference points at
a non-existent ``ms.persistence``), and /set values keep their case.

Console script: ``lazzaro-amd-cli`` (``python -m lazzaro_amd.cli.main``).
"""
from __future__ import annotations

import argparse
import os

CONFIG_KEYS = ("max_buffer_size", "prune_threshold", "consolidate_every", "auto_consolidate", "auto_prune",
               "enable_sharding", "enable_hierarchy", "enable_caching", "enable_async")
HELP = ("Available commands: /start, /end, /stats, /profile, /memories [n], /consolidate, /merge, "
        "/prune [thresh], /config, /set <k> <v>, /save [file], /load [file], /quit")


def _coerce(cur, raw: str):
    if isinstance(cur, bool):
        return raw.lower() in ("true", "1", "on", "yes")
    return type(cur)(raw)


def handle_command(memory, line: str, out=print) -> bool:
    """Execute one slash command; returns False when the REPL should exit."""
    parts = line.split()
    cmd = parts[0].lower()
    if cmd == "/quit":
        if memory.conversation_active:
            out("\n" + memory.end_conversation())
        memory.flush()
        out("\n👋 Goodbye!")
        return False
    if cmd == "/start":
        out("\n" + memory.start_conversation())
    elif cmd == "/end":
        out("\n" + memory.end_conversation())
    elif cmd == "/stats":
        out(memory.display_stats())
    elif cmd == "/profile":
        out(memory.display_profile())
    elif cmd == "/memories":
        out(memory.display_memories(limit=int(parts[1]) if len(parts) > 1 else 10))
    elif cmd == "/consolidate":
        out("\n" + memory.run_consolidation())
    elif cmd == "/merge":
        out("\n🔄 Merging similar nodes...")
        out(f"✓ Merged {memory._merge_similar_nodes()} similar nodes")
    elif cmd == "/prune":
        thr = float(parts[1]) if len(parts) > 1 else memory.prune_threshold
        out(f"\n🔄 Pruning edges below {thr}...")
        out(f"✓ Pruned {memory.buffer.prune_weak_edges(threshold=thr)} weak edges")
    elif cmd == "/config":
        out("\n⚙️ Configuration:")
        for k in CONFIG_KEYS:
            out(f"  • {k}: {getattr(memory, k)}")
    elif cmd == "/set":
        if len(parts) < 3:
            out("⚠ Usage: /set <parameter> <value>")
        elif not hasattr(memory, parts[1]):
            out(f"⚠ Unknown parameter: {parts[1]}")
        else:
            try:
                val = _coerce(getattr(memory, parts[1]), parts[2])
                setattr(memory, parts[1], val)
                out(f"✓ Set {parts[1]} = {val}")
            except ValueError:
                out(f"⚠ Invalid value for {parts[1]}")
    elif cmd == "/save":
        memory._save_to_persistence()
        fn = parts[1] if len(parts) > 1 else "memory_state.json"
        out("\n" + memory.save_state(fn))
        out(f"✓ Also persisted to the store at {getattr(memory.store, 'db_dir', '?')}")
    elif cmd == "/load":
        if len(parts) > 1:
            out("\n" + memory.load_state(parts[1]))
        else:
            memory._load_from_persistence()
            out(f"\n✓ Reloaded from the store at {getattr(memory.store, 'db_dir', '?')}")
    elif cmd == "/help":
        out(HELP)
    else:
        out(f"⚠ Unknown command {cmd}. {HELP}")
    return True


def interactive_chat(memory=None, input_fn=input, out=print) -> None:
    if memory is None:
        from ..core.memory_system import MemorySystem

        memory = MemorySystem(os.environ.get("OPENAI_API_KEY"), enable_sharding=True, enable_hierarchy=True,
                              enable_caching=True, enable_async=True, max_buffer_size=10, prune_threshold=0.5)
    out("=" * 60)
    out("  SCALABLE MEMORY SYSTEM - CLI (MI355X engine)")
    out("=" * 60)
    out("\nCommands: /start, /end, /stats, /profile, /memories, /consolidate")
    out("          /merge, /prune, /config, /set, /save, /load, /quit")
    while True:
        try:
            line = input_fn("\nYou: ").strip()
        except (KeyboardInterrupt, EOFError):
            out("\n👋 Goodbye!")
            break
        if not line:
            continue
        try:
            if line.startswith("/"):
                if not handle_command(memory, line, out):
                    break
                continue
            if out is print:
                print("Assistant: ", end="", flush=True)
            toks = []
            for ev in memory.chat_stream(line):
                if ev["type"] == "info" and not toks:
                    out(f"\n{ev['content']}")
                elif ev["type"] == "token":
                    toks.append(ev["content"])
                    if out is print:
                        print(ev["content"], end="", flush=True)
            if out is not print:
                out("Assistant: " + "".join(toks))
            else:
                print()
        except Exception as e:  # keep the REPL alive
            out(f"\n⚠ Error: {e}")


def entry_point() -> None:
    ap = argparse.ArgumentParser(description="lazzaro_amd interactive memory CLI")
    ap.add_argument("--db-dir", default="db")
    ap.add_argument("--user", default="default")
    a = ap.parse_args()
    from ..core.memory_system import MemorySystem

    ms = MemorySystem(os.environ.get("OPENAI_API_KEY"), db_dir=a.db_dir, user_id=a.user, verbose=True)
    interactive_chat(ms)
    ms.close()


if __name__ == "__main__":
    entry_point()
