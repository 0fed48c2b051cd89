"""Refresh the code blocks of INTEGRATION.md that follow an
`<!-- embed: path -->` marker with the current contents of that file
(integration/go/*).  tests/test_integration_go.py checks they agree."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"(<!-- embed: (\S+) -->\n```(\w*)\n)(.*?)(```\n)", re.S)


def render(text):
    def sub(m):
        with open(os.path.join(ROOT, m.group(2))) as f:
            body = f.read()
        if not body.endswith("\n"):
            body += "\n"
        return m.group(1) + body + m.group(5)
    return PAT.sub(sub, text)


if __name__ == "__main__":
    p = os.path.join(ROOT, "INTEGRATION.md")
    with open(p) as f:
        old = f.read()
    new = render(old)
    if "--check" in sys.argv:
        sys.exit(0 if new == old else 1)
    with open(p, "w") as f:
        f.write(new)
