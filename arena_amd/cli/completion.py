"""bash/zsh completion scripts generated from the argparse tree (the reference's `completion`
command existed but was never registered -- completion.go:12-49, root.go:35; registered here)."""
from __future__ import annotations

import argparse


def _tree(parser: argparse.ArgumentParser, prefix=()):
    cmds = {}
    for a in parser._actions:  # noqa: SLF001
        if isinstance(a, argparse._SubParsersAction):  # noqa: SLF001
            for name, sp in a.choices.items():
                cmds[prefix + (name,)] = sp
                cmds.update(_tree(sp, prefix + (name,)))
    return cmds


def _flags(parser) -> list:
    out = []
    for a in parser._actions:  # noqa: SLF001
        out += [o for o in a.option_strings if o.startswith("--")]
    return sorted(set(out))


def completion_script(shell: str, parser) -> str:
    tree = _tree(parser)
    top = sorted({k[0] for k in tree})
    cases = []
    for path, sp in sorted(tree.items()):
        subs = sorted({k[len(path)] for k in tree if len(k) == len(path) + 1 and k[:len(path)] == path})
        words = " ".join(subs + _flags(sp))
        cases.append((" ".join(path), words))
    if shell == "bash":
        body = "\n".join(f'        "{p}") opts="{w}" ;;' for p, w in cases)
        return f'''# bash completion for arena
_arena() {{
    local cur path opts
    cur="${{COMP_WORDS[COMP_CWORD]}}"
    path="${{COMP_WORDS[*]:1:COMP_CWORD-1}}"
    opts="{' '.join(top + _flags(parser))}"
    case "$path" in
{body}
    esac
    COMPREPLY=( $(compgen -W "$opts" -- "$cur") )
}}
complete -F _arena arena
'''
    body = "\n".join(f'    "{p}") opts=({w}) ;;' for p, w in cases)
    return f'''#compdef arena
_arena() {{
  local -a opts
  local path="${{words[2,CURRENT-1]}}"
  opts=({' '.join(top + _flags(parser))})
  case "$path" in
{body}
  esac
  compadd -- $opts
}}
compdef _arena arena
'''
