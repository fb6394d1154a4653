"""The tree stays lint-clean (tools/lint.py; the reference CI lints with
pycodestyle + flake8, ``/root/reference/.travis.yml:31-32``)."""
import os.path as osp
import sys

sys.path.insert(0, osp.join(osp.dirname(osp.dirname(__file__)), 'tools'))
import lint  # noqa: E402


def test_repository_is_lint_clean():
    findings = lint.lint()
    assert not findings, '\n'.join('{}:{}: {}'.format(*f)
                                   for f in findings[:50])


def test_lint_catches_violations(tmp_path):
    bad = tmp_path / 'bad.py'
    bad.write_text('import os\nx = 1 \n' + 'y = "' + 'a' * 80 + '"\n')
    codes = {m.split()[0] for _, _, m in lint.lint([str(bad)])}
    assert {'F401', 'W291', 'E501'} <= codes
    hip = tmp_path / 'k.hip'
    hip.write_text('#ifdef __HIP_PLATFORM_AMD__\n#endif\n')
    assert any('X001' in m for _, _, m in lint.lint([str(hip)]))
